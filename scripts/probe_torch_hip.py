"""Does torch's HIP runtime coexist with libemqx_gpu_match.so in one process?
Each scenario runs in its own subprocess: A torch first, B the library first,
C an RCCL process group (world 1) + all_reduce on a device tensor, then the
library.  Prints one line per scenario."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRE = f"import sys; sys.path.insert(0, {ROOT!r}); import numpy as np\n"
MATCH = """
from emqx_amd import Context
with Context(0) as ctx:
    idx = ctx.build_index([b'a/+', b'a/#', b'b'])
    ro, ids = ctx.match(idx, [b'a/x', b'b', b'c'])
    assert ro.tolist() == [0, 2, 3, 3], ro
    idx.release()
"""
TORCH = """
import torch
x = torch.ones(1024, device='cuda:0'); assert float(x.sum()) == 1024.0
"""
RCCL = """
import torch, torch.distributed as dist
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT='29533', RANK='0', WORLD_SIZE='1')
torch.cuda.set_device(0)
dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
t = torch.ones(8, device='cuda:0'); dist.all_reduce(t); assert float(t.sum()) == 8.0
"""
scen = {"A_torch_then_lib": TORCH + MATCH, "B_lib_then_torch": MATCH + TORCH,
        "C_rccl_then_lib": "import os\n" + RCCL + MATCH + "dist.destroy_process_group()\n"}
for name, code in scen.items():
    p = subprocess.run([sys.executable, "-c", PRE + code], capture_output=True, text=True, timeout=240)
    print(name, "rc", p.returncode, (p.stderr.strip().splitlines() or [""])[-1][:300], flush=True)
