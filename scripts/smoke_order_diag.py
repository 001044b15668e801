"""Which HIP runtime the library and torch end up on, by process order
(diagnostic for the round-5 smoke failure: emqx_gm_open EDEVICE when a host-only
library call came before the first Context; run by
tests/test_gpu_sharded.py::test_one_hip_runtime_whatever_the_order).
usage: smoke_order_diag.py MODE
  lib_first    a host-only library call (gen_filter_codes), then Context(0)
  torch_first  import torch, then the same
  ctx_first    Context(0) first"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def maps():
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if "amdhip64" in ln or "hsa-runtime" in ln})


mode = sys.argv[1]
if mode == "torch_first":
    import torch  # noqa: F401
from emqx_amd import Context  # noqa: E402
from emqx_amd.engine import gen_filter_codes  # noqa: E402

if mode != "ctx_first":
    gen_filter_codes(1, 100)
print(mode, "loaded:", maps(), flush=True)
try:
    with Context(0) as ctx:
        print(mode, "open ok", ctx.devices, flush=True)
except Exception as e:  # noqa: BLE001
    print(mode, "open FAILED:", e, flush=True)
import torch  # noqa: E402

print(mode, "torch available:", torch.cuda.is_available(), "maps:", maps(), flush=True)
print(mode, "hip runtimes:", sum("amdhip64" in m for m in maps()), flush=True)
