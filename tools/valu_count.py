"""Static instruction counts of the library's gfx950 kernels.

Unbundles the device code object of each cuda-dct-idct_amd/build/*.o
(clang-offload-bundler), disassembles it (llvm-objdump) and counts, per
kernel symbol, the VALU (v_*, of which packed v_pk_*), SALU (s_*), vector
memory (global_* / buffer_*) and LDS (ds_*) instructions.  The tile kernels
are straight-line per 64-tile set (one set per wave), so the static VALU count
is the per-wave count SQ_INSTS_VALU / SQ_WAVES measures on the GPU.

  python3 tools/valu_count.py [filter-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "cuda-dct-idct_amd", "build")
LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    with tempfile.TemporaryDirectory() as d:
        co, fat = os.path.join(d, "k.co"), os.path.join(d, "fat.bin")
        r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj,
                            os.path.join(d, "host.o")], capture_output=True, text=True)
        if r.returncode != 0:
            return ""
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}",
                            "--unbundle"], capture_output=True, text=True)
        if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
            return ""
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                              text=True).stdout


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.split("\n") if r.returncode == 0 else names


def counts(text):
    out = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] = {"valu": 0, "pk": 0, "salu": 0, "vmem": 0, "lds": 0, "total": 0}
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+([a-z_0-9]+)", line)
        if not m:
            continue
        op = m.group(1)
        c = out[cur]
        c["total"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
            if op.startswith("v_pk_"):
                c["pk"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith(("global_", "buffer_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    return out


def main(filters):
    rows = []
    for f in sorted(os.listdir(BUILD)):
        if not f.endswith(".o"):
            continue
        res = counts(disasm(os.path.join(BUILD, f)))
        names = list(res)
        for raw, dm in zip(names, demangle(names)):
            if filters and not all(s in dm for s in filters):
                continue
            rows.append((f, dm, res[raw]))
    for f, dm, c in rows:
        print(f"{c['valu']:6d} valu ({c['pk']:4d} pk) {c['salu']:5d} salu {c['vmem']:4d} vmem {c['lds']:4d} lds  "
              f"{f}: {dm}")


if __name__ == "__main__":
    main(sys.argv[1:])
