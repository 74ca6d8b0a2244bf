"""Time float64 flooding-kernel variants (build/fdev/*.so) beside the product library on the same
LLRs and check each bit-exact against it (development tool, not product).

    python tools/flood_dev/run_dev.py build/fdev/base.so build/fdev/noB.so ...
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402

ZC, K, N, NF = 384, 22 * 384, 66 * 384, 68 * 384


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    B = int(os.environ.get("FDEV_B", "4096"))
    snrs = [float(x) for x in os.environ.get("FDEV_SNR", "-3,0.5").split(",")]
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, 1)
    libs = [(p, ctypes.CDLL(os.path.abspath(p))) for p in sys.argv[1:]]
    for snr in snrs:
        sigma = 10 ** (-snr / 20)
        llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, device="cuda", dtype=torch.float64,
                                                                  generator=g)) / sigma ** 2).contiguous()
        dead = int(os.environ.get("FDEV_DEADCOLS", "0"))   # the last `dead` extension columns untransmitted
        if dead:
            llr[:, -dead * ZC:] = 0.0
        ref = (torch.empty((B, NF), dtype=torch.int8, device="cuda"), torch.empty((B,), dtype=torch.uint8, device="cuda"),
               torch.empty((B,), dtype=torch.int32, device="cuda"))
        prod = lambda: D.nr_decode_ldpc_batch(llr, ZC, 1, 8, "min-sum", 0.75, 0.0, "flooding", out=ref,  # noqa: E731
                                              rate_matched=bool(dead))
        runs = [("product", prod)]
        outs = {}
        for p, lib in libs:
            out = (torch.full((B, NF), 7, dtype=torch.int8, device="cuda"), torch.full((B,), 9, dtype=torch.uint8, device="cuda"),
                   torch.full((B,), -1, dtype=torch.int32, device="cuda"))
            st = torch.cuda.current_stream().cuda_stream

            def run(lib=lib, out=out):
                rc = lib.fdev_decode(ctypes.c_void_p(llr.data_ptr()), ctypes.c_void_p(out[0].data_ptr()),
                                     ctypes.c_void_p(out[1].data_ptr()), ctypes.c_void_p(out[2].data_ptr()),
                                     B, ZC, ctypes.c_longlong(N), ctypes.c_longlong(NF), 8,
                                     ctypes.c_double(0.75), ctypes.c_void_p(st))
                assert rc == 0, rc
            runs.append((os.path.basename(p), run))
            outs[os.path.basename(p)] = out
        # interleaved rounds, median per variant (single runs vary by ~2 %)
        times = {n: [] for n, _ in runs}
        for _ in range(int(os.environ.get("FDEV_ROUNDS", "5"))):
            for n, fn in runs:
                times[n].append(timeit(fn))
        for n, _ in runs:
            t = sorted(times[n])
            ms = t[len(t) // 2]
            extra = ""
            if n == "product":
                extra = f"  iters {ref[2].float().mean().item():.2f}"
            else:
                extra = f"  exact={all(torch.equal(a, b) for a, b in zip(outs[n], ref))}"
            print(f"snr {snr}: {n}: median {ms:.3f} ms ({B / ms / 1e3:.3f} M CB/s) min {t[0]:.3f} max {t[-1]:.3f}{extra}",
                  flush=True)

if __name__ == "__main__":
    main()
