"""HBM ceiling for the encoder's traffic mix (development tool): torch kernels that read 8,448 B
and write 25,344 B per codeblock (the BG1 Zc=384 encoder's algorithmic bytes), beside a pure
write (fill) and a 1:1 copy, at 16384 codeblocks (553 MB, past the 256 MB MALL).

    python tools/bw_mix_probe.py [B]
"""
import sys

import torch


def timeit(fn, reps=30):
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    K, N = 8448, 25344
    ck = torch.randint(0, 2, (B, K), dtype=torch.int8, device="cuda")
    dn = torch.empty((B, N), dtype=torch.int8, device="cuda")
    ms = timeit(lambda: dn.fill_(1))
    print(f"fill {B}x{N} B: {ms * 1e3:.1f} us  {B * N / ms / 1e6:.0f} GB/s (write only)")
    big = torch.empty((B, K * 2), dtype=torch.int8, device="cuda")
    src = torch.randint(0, 2, (B, K * 2), dtype=torch.int8, device="cuda")
    ms = timeit(lambda: big.copy_(src))
    print(f"copy {B}x{2 * K} B: {ms * 1e3:.1f} us  {2 * B * 2 * K / ms / 1e6:.0f} GB/s (read+write 1:1)")
    v = dn.view(B, 3, K)
    ms = timeit(lambda: v.copy_(ck.unsqueeze(1).expand(B, 3, K)))
    print(f"expand-copy read {K} write {N} per row: {ms * 1e3:.1f} us  {B * (K + N) / ms / 1e6:.0f} GB/s")
    c32 = ck.view(torch.int32)
    d32 = dn.view(torch.int32).view(B, 3, K // 4)
    ms = timeit(lambda: d32.copy_(c32.unsqueeze(1).expand(B, 3, K // 4)))
    print(f"expand-copy int32 view: {ms * 1e3:.1f} us  {B * (K + N) / ms / 1e6:.0f} GB/s")


if __name__ == "__main__":
    main()
