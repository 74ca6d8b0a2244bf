"""Throughput probes (development tool, not the bench contract): time the encoder / decoders
over several batch sizes with HIP events.

    python tools/probe.py encode 1024 4096 16384 65536
    python tools/probe.py layered 1024 4096 8192
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E  # noqa: E402

BG = int(os.environ.get("PROBE_BG", "1"))
ZC = 384
K, N, NF = ((22, 66, 68) if BG == 1 else (10, 50, 52))
K, N, NF = K * ZC, N * ZC, NF * ZC


def timeit(fn, reps):
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
    what = sys.argv[1]
    if what == "occupancy":
        from python_5gtoolbox_amd import _lib
        lib = _lib.lib()
        for bg in (1, 2):
            for name, dt, sch in (("f64 flooding", 0, 0), ("f32 flooding", 1, 0), ("f32 layered", 1, 1)):
                print(f"BG{bg} {name}: {lib.ldpc5g_dec_blocks_per_cu(bg, dt, sch)} workgroups/CU")
        return
    sizes = [int(x) for x in sys.argv[2:]] or [4096]
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    for B in sizes:
        ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda", generator=g)
        if what == "encode":
            dn = torch.empty((B, N), dtype=torch.int8, device="cuda")
            ms = timeit(lambda: E.encode_ldpc_batch(ck, BG, out=dn), 50)
            print(f"encode B={B}: {ms * 1e3:.1f} us  {B / ms / 1e3:.1f} M CB/s  "
                  f"{B * (K + N) / ms / 1e6:.0f} GB/s")
        else:
            dn = E.encode_ldpc_batch(ck, BG)
            sigma = 10 ** (-float(os.environ.get("PROBE_SNR", "-3")) / 20)   # default -3 dB
            llr = (2 * ((1 - 2 * dn.float()) + sigma * torch.randn(dn.shape, device="cuda",
                                                                     generator=g)) / sigma ** 2)
            out = (torch.empty((B, NF), dtype=torch.int8, device="cuda"),
                   torch.empty((B,), dtype=torch.uint8, device="cuda"),
                   torch.empty((B,), dtype=torch.int32, device="cuda"))
            sched = what
            if what == "flooding64":   # the reference-exact float64 flooding mode
                llr, sched = llr.double(), "flooding"
            L = int(os.environ.get("PROBE_L", "8"))
            ms = timeit(lambda: D.nr_decode_ldpc_batch(llr, ZC, BG, L, "min-sum", 0.75, 0.0, sched,
                                                       out=out), 5)
            print(f"{what} L={L} B={B}: {ms:.3f} ms  {B / ms / 1e3:.3f} M CB/s  iters "
                  f"{out[2].float().mean().item():.2f}")


if __name__ == "__main__":
    main()
