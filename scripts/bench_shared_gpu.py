"""Rehearsal of bench.py's N>1 path on a one-GPU box: every rank that
torch.distributed.run starts maps to device 0 (LOCAL_RANK=0), so the weight
broadcast, the gloo barriers, the settle period and the timed region run as
in an N-GPU job (the ranks share the card).  RCCL refuses two ranks on one
device, so the post-region exchange needs DSTD_BENCH_BACKEND=gloo here."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["LOCAL_RANK"] = "0"
import bench  # noqa: E402

bench.main()
