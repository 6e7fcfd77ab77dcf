"""HIP device attributes the launch code relies on (hpdct_launch.hpp:
device_cus(), device_lds_per_cu()), read through the same hipDeviceGetAttribute
calls, plus torch's view of the device.  Run on the GPU box
(tools/gpu_session.sh ... devinfo)."""
import ctypes
import json

import torch

ATTRS = {  # hipDeviceAttribute_t values (hip/hip_runtime_api.h, ROCm 7.2)
    "hipDeviceAttributeMultiprocessorCount": None,
    "hipDeviceAttributeMaxSharedMemoryPerMultiprocessor": None,
    "hipDeviceAttributeMaxSharedMemoryPerBlock": None,
    "hipDeviceAttributeSharedMemPerBlockOptin": None,
}


def main():
    torch.cuda.init()
    p = torch.cuda.get_device_properties(0)
    lib = ctypes.CDLL("libamdhip64.so.7")
    # attribute enum values, from a tiny query of the header-defined names
    import os
    import subprocess
    import tempfile
    src = "#include <hip/hip_runtime.h>\n#include <stdio.h>\nint main(){printf(\"%d %d %d %d\\n\"," + ",".join(
        f"(int){a}" for a in ATTRS) + ");}\n"
    vals = None
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "a.cpp")
        open(c, "w").write(src)
        exe = os.path.join(d, "a")
        r = subprocess.run(["/opt/rocm/bin/hipcc", c, "-o", exe], capture_output=True, text=True)
        if r.returncode == 0:
            vals = [int(v) for v in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    out = {"torch_name": p.name, "torch_multi_processor_count": p.multi_processor_count,
           "gcnArchName": getattr(p, "gcnArchName", None)}
    if vals:
        for name, code in zip(ATTRS, vals):
            v = ctypes.c_int()
            rc = lib.hipDeviceGetAttribute(ctypes.byref(v), code, 0)
            out[name] = v.value if rc == 0 else f"error {rc}"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
