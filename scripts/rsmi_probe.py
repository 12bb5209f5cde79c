"""Probe for the RCCL-alive slowdown: does initialising the ROCm
SMI library in the process (RCCL's topology detection does) slow the forward?
Runs bench.main() after rsmi_init(0) (librocm_smi64) or amdsmi_init
(libamd_smi), per argv[1] in {rsmi, amdsmi, none}; the rest of argv goes to
bench.py."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

mode = sys.argv.pop(1)
if mode == "rsmi":
    lib = ctypes.CDLL("/opt/rocm/lib/librocm_smi64.so")
    print("rsmi_init", lib.rsmi_init(ctypes.c_uint64(0)), file=sys.stderr)
elif mode == "amdsmi":
    lib = ctypes.CDLL("/opt/rocm/lib/libamd_smi.so")
    print("amdsmi_init", lib.amdsmi_init(ctypes.c_uint64(2)), file=sys.stderr)  # AMDSMI_INIT_AMD_GPUS
import bench  # noqa: E402

bench.main()
