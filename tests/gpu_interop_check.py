"""Developer diagnostic: torch (imported first) and libhsddp_amd.so share one HIP runtime."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hkd-mpc_amd"))
import hsddp
from hsddp._lib import lib, check
x = torch.rand(128, 24, dtype=torch.float64, device="cuda"); x[:, 5] += 0.2
u = torch.rand(128, 24, dtype=torch.float64, device="cuda")
c = torch.ones(128, 4, dtype=torch.float64, device="cuda")
xn = torch.empty_like(x)
check(lib().hsddp_hkd_dynamics(x.data_ptr(), u.data_ptr(), c.data_ptr(), 0.01, xn.data_ptr(), 128,
                               torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
ref = hsddp.model.dynamics(x.cpu().numpy(), u.cpu().numpy(), c.cpu().numpy())
print("interop max err", float((xn.cpu() - torch.from_numpy(ref)).abs().max()))
import subprocess
maps = open(f"/proc/{os.getpid()}/maps").read()
print("amdhip64 copies:", sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l}))
