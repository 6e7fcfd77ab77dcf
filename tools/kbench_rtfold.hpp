// kbench_rtfold.hpp -- round 6 A/B (tools/kb_rt group "fold"): the C3 round
// trip with the sums fold inside the round-trip kernel, instead of the
// product's second one-wave dispatch (rt_spread_finish_kernel).  Measured and
// rejected: 74.9-75.1 us against 73.8-74.6 for the product at 8192^2, both
// bit-exact (profiles/r06/kb_rt_fold.log): the returning atomics every wave
// needs before its ticket cost more than the fold kernel's dispatch saves.
#pragma once

#include "hpdct_rt_duo.hpp"

namespace hpdct {

// The same round trip with the fold inside the kernel (no second dispatch):
// the waves' tickets find the last wave, which folds the spread slot into
// *out itself.  Each wave's lane 0 adds its sums into sub-slot k = wave % 64
// with RETURNING atomics (performed at the device's coherence point once they
// return) and only then takes sub-slot k's ticket (word kTicketWord of the
// sub-slot, on its second 128-B line); the wave that takes the sub-slot's last
// ticket resets it and takes the global ticket (sub-slot 0, word
// kGlobalWord); the wave that takes the last global ticket has seen every
// wave's sums performed, so it takes the 64 sub-slots with atomic exchanges
// (zeroing them), resets the global ticket and writes *out (overwrite) or
// adds to it with atomics (accumulate).  Two levels of tickets keep each
// ticket line at <= nwaves / 64 atomics.  The slot must not be shared by two
// launches in flight (the launcher keys it by stream as well as pointer).
constexpr uint32_t kTicketWord = 16, kGlobalWord = 24;
template <bool kStats, int kQMode, int kRecon, int kBlockT = 256, int kWaves = 6>
__global__ __launch_bounds__(kBlockT) __attribute__((amdgpu_waves_per_eu(kWaves, 8))) void roundtrip_duo_fold_kernel(
    const uint8_t* __restrict__ img, float* __restrict__ coef, void* __restrict__ recon,
    unsigned long long* __restrict__ spread, RtSums* __restrict__ out, TileGrid g, QParams qp, int accumulate) {
    static_assert(kStats, "the fold kernel exists for the sums");
    constexpr uint32_t kW = kBlockT / 64u;
    uint32_t wave;
    const DuoWaveSums w = rt_duo_waves<true, kQMode, kRecon, true, kBlockT, 1>(img, coef, recon, g, qp, wave);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nwaves = gridDim.x * kW;
    const uint32_t k = wave % static_cast<uint32_t>(kRtSpread);
    const uint32_t in_k = nwaves / kRtSpread + (k < nwaves % kRtSpread ? 1u : 0u);   // waves of sub-slot k
    const uint32_t used = nwaves < static_cast<uint32_t>(kRtSpread) ? nwaves : kRtSpread;  // non-empty sub-slots
    uint32_t last = 0u;
    if (lane == 0u) {
        uint32_t z = 0u;
        asm volatile("" : "+v"(z));
        unsigned long long* const sub = spread + k * kRtSpreadStride + z;
        const unsigned long long a0 = atomicAdd(sub, w.fs), a1 = atomicAdd(sub + 1, static_cast<unsigned long long>(w.se)),
                                 a2 = atomicAdd(sub + 2, static_cast<unsigned long long>(w.sx));
        const unsigned long long a3 = w.bad ? atomicOr(sub, kRtSseF32Invalid) : 0ull;
        // the tickets go out only once the sums have returned (the returned
        // values feed the asm, which the ticket atomic follows)
        const unsigned long long dep = a0 ^ a1 ^ a2 ^ a3;
        asm volatile("" ::"v"(dep) : "memory");
        unsigned int* const tk = reinterpret_cast<unsigned int*>(sub + kTicketWord);
        if (atomicAdd(tk, 1u) == in_k - 1u) {
            atomicExch(tk, 0u);  // sub-slot k complete: reset for the next launch
            unsigned int* const gt = reinterpret_cast<unsigned int*>(spread + kGlobalWord + z);
            if (atomicAdd(gt, 1u) == used - 1u) {
                atomicExch(gt, 0u);
                last = 1u;
            }
        }
    }
    if (__builtin_amdgcn_readfirstlane(last) == 0u) return;
    // the last wave: lane l takes sub-slot l (and zeroes it)
    unsigned long long v[3], bad[3];
    unroll<3>([&](auto f) {
        const unsigned long long x = atomicExch(&spread[lane * kRtSpreadStride + f], 0ull);
        v[f] = x & ~kRtSseF32Invalid, bad[f] = x & kRtSseF32Invalid;
    });
    unroll<3>([&](auto f) {
        const unsigned long long sum = wave_sum_dpp(v[f]);
        const bool flagged = __builtin_amdgcn_ballot_w64(bad[f] != 0ull) != 0ull;
        if (lane == 0u) {
            auto* const d = reinterpret_cast<unsigned long long*>(out) + f;
            if (accumulate) {
                if (sum) atomicAdd(d, sum);
                if (flagged) atomicOr(d, kRtSseF32Invalid);
            } else {
                *d = flagged ? (sum | kRtSseF32Invalid) : sum;
            }
        }
    });
}

}  // namespace hpdct
