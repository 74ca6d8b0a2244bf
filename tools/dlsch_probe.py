"""Where the DLSCHDecode drop-in's time goes for one 23-codeblock TB (dev tool)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from python_5gtoolbox_amd import nr_dlsch, nr_dlsch_decode  # noqa: E402
from python_5gtoolbox_amd.sch import sch_config, sch_decode_batch  # noqa: E402

A, Qm, R, NL, rv, LBRM, G = 193728, 8, 700, 2, 0, 1081512, 278016
dec = {"L": 8, "algo": "min-sum", "alpha": 0.75, "beta": 0.0}
rng = np.random.default_rng(1)
tb = rng.integers(0, 2, A).astype(np.int8)
g = nr_dlsch.DLSCHEncode(tb, A, Qm, R, NL, rv, LBRM, G)
llr = (1 - 2 * g.astype(np.float64)) * 20.0 + rng.normal(0, 0.5, G)
for _ in range(3):
    nr_dlsch_decode.DLSCHDecode(llr, A, Qm, R, NL, rv, LBRM, dec)
torch.cuda.synchronize()


def t(fn, n=10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, r


cfg = sch_config(A, Qm, R, NL, rv, LBRM, G)
print("whole DLSCHDecode ms", t(lambda: nr_dlsch_decode.DLSCHDecode(llr, A, Qm, R, NL, rv, LBRM, dec))[0])
print("sch_config ms", t(lambda: sch_config(A, Qm, R, NL, rv, LBRM, G))[0])
x = torch.from_numpy(llr.reshape(1, -1)).cuda()
print("H2D ms", t(lambda: torch.from_numpy(llr.reshape(1, -1)).cuda())[0])
ms, r = t(lambda: sch_decode_batch(x, cfg, 8, "min-sum", 0.75, 0.0, "flooding", None, torch.float64))
print("sch_decode_batch (device, sync) ms", ms)
print("D2H llr_dn ms", t(lambda: r.llr_dn.cpu().numpy())[0])
print("D2H tbblk+ok ms", t(lambda: (r.tbblk[0, :A].cpu().numpy(), r.tb_ok.cpu().numpy()))[0])
print("mean iterations", r.iters.float().mean().item())

from python_5gtoolbox_amd import _lib  # noqa: E402
from python_5gtoolbox_amd.sch import SchWorkspace  # noqa: E402


def steps():
    tt = [time.perf_counter()]
    t_ = _lib.require_gpu(); tt.append(time.perf_counter())
    ll = np.ascontiguousarray(np.asarray(llr, np.float64).reshape(1, -1)); tt.append(time.perf_counter())
    xx = t_.from_numpy(ll).cuda(); tt.append(time.perf_counter())
    ws = SchWorkspace(cfg, 1, xx.device); tt.append(time.perf_counter())
    rr = sch_decode_batch(xx, cfg, 8, "min-sum", 0.75, 0.0, "flooding", None, torch.float64, ws); tt.append(time.perf_counter())
    ok = bool(rr.tb_ok.cpu().numpy()[0]); tt.append(time.perf_counter())
    blk = rr.tbblk[0, :cfg.A].cpu().numpy().astype("i1"); tt.append(time.perf_counter())
    new = rr.llr_dn.cpu().numpy().astype(np.float64); tt.append(time.perf_counter())
    return np.diff(tt) * 1e3


for _ in range(3):
    steps()
acc = np.mean([steps() for _ in range(10)], axis=0)
print("require_gpu, asarray, H2D, workspace, decode(async), tb_ok D2H(sync), tbblk D2H, llr_dn D2H (ms):",
      np.round(acc, 3))
