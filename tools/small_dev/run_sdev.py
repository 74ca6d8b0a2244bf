"""Time small-codeblock decoder builds (build/sdev/*.so) beside the product on one BG2 Zc=8
codeblock (BASELINE config 1 shape) and check them bit-exact; a *_ts.so build prints thread 0's
phase timestamps (cycles) instead (development tool, not product).

    python tools/small_dev/run_sdev.py build/sdev/base.so build/sdev/base_ts.so
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402
from python_5gtoolbox_amd.ldpc_info import code_dims  # noqa: E402


def timeit(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    libs = [(p, ctypes.CDLL(os.path.abspath(p))) for p in sys.argv[1:]]
    for bg, Zc, B in [(2, 8, 1), (1, 8, 1), (2, 32, 1)]:
        K, N, Nf = code_dims(bg, Zc)
        ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
        dn = E.encode_ldpc_batch(ck, bg)
        sigma = 10 ** (3 / 20)
        llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, dtype=torch.float64, device="cuda",
                                                                  generator=g)) / sigma ** 2).contiguous()
        ref = (torch.empty((B, Nf), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
               torch.empty((B,), dtype=torch.int32, device="cuda"))
        us = timeit(lambda: D.nr_decode_ldpc_batch(llr, Zc, bg, 8, "min-sum", 0.75, 0.0, "flooding", out=ref))
        print(f"BG{bg} Zc={Zc} B={B}: product {us:.1f} us/call iters {ref[2].float().mean().item():.2f}", flush=True)
        for p, lib in libs:
            out = (torch.full((B, Nf), 7, dtype=torch.int8, device="cuda"), torch.full((B,), 9, dtype=torch.uint8, device="cuda"),
                   torch.full((B,), -1, dtype=torch.int32, device="cuda"))
            st = torch.cuda.current_stream().cuda_stream

            def run():
                rc = lib.sdev_decode(bg, ctypes.c_void_p(llr.data_ptr()), ctypes.c_void_p(out[0].data_ptr()),
                                     ctypes.c_void_p(out[1].data_ptr()), ctypes.c_void_p(out[2].data_ptr()),
                                     B, Zc, ctypes.c_longlong(N), ctypes.c_longlong(Nf), 8,
                                     ctypes.c_double(0.75), ctypes.c_void_p(st))
                assert rc == 0, rc
            us = timeit(run)
            if p.endswith("_ts.so"):
                run()
                torch.cuda.synchronize()
                ts = out[0][0, :128].cpu().view(torch.int64).tolist()
                d = [ts[i] - ts[0] if ts[i] else None for i in range(16)]
                print(f"  {os.path.basename(p)}: {us:.1f} us/call  stamps(cycles from start) {d}", flush=True)
            else:
                same = all(torch.equal(a, b) for a, b in zip(out, ref))
                print(f"  {os.path.basename(p)}: {us:.1f} us/call exact={same}", flush=True)


if __name__ == "__main__":
    main()
