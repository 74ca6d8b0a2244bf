"""Two (or more) processes on one GPU, each launching the multi-workgroup float64 decoder
(ldpc5g_dec_split.hip) back to back with 12 BG1 Zc=384 codeblocks (216 workgroups per launch, so
two processes' launches cannot be resident together): the ticket-ordered parts must let both finish.
Each child checks every repetition against its first.  Development tool / gpu test helper.

    python tools/split_mp_probe.py [procs] [reps]          (parent)
    python tools/split_mp_probe.py --child SEED REPS       (one process)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(seed, reps):
    import torch
    from python_5gtoolbox_amd import nr_ldpc_decode as D, nr_ldpc_encode as E
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    B, Zc = 12, 384
    ck = torch.randint(0, 2, (B, 22 * Zc), dtype=torch.int8, device="cuda", generator=g)
    dn = E.encode_ldpc_batch(ck, 1)
    sigma = 10 ** (-1.0 / 20)
    llr = (2 * ((1 - 2 * dn.double()) + sigma * torch.randn(dn.shape, dtype=torch.float64, device="cuda",
                                                              generator=g)) / sigma ** 2).contiguous()
    ref = [t.clone() for t in D.nr_decode_ldpc_batch(llr, Zc, 1, 8, "min-sum", 0.75, 0.0, "flooding")]
    torch.cuda.synchronize()
    print("ready", flush=True)   # the parent starts every child's timed loop at once
    sys.stdin.readline()
    t0 = time.time()
    outs = [D.nr_decode_ldpc_batch(llr, Zc, 1, 8, "min-sum", 0.75, 0.0, "flooding") for _ in range(reps)]
    torch.cuda.synchronize()
    dt = time.time() - t0
    bad = sum(not all(torch.equal(a, b) for a, b in zip(o, ref)) for o in outs)
    print(f"child {seed}: {reps} launches in {dt * 1e3:.1f} ms, mismatches {bad}", flush=True)
    return 1 if bad else 0


def main():
    if sys.argv[1:2] == ["--child"]:
        sys.exit(child(int(sys.argv[2]), int(sys.argv[3])))
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    # the children stay in this process's group: a caller that starts this probe in a session of
    # its own (tests/test_gpu_ldpc.py) kills them all with it on a time limit
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", str(11 + k), str(reps)],
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
          for k in range(procs)]
    deadline = time.time() + 120
    try:
        for p in ps:   # every child warmed up, then all go together
            line = p.stdout.readline()
            assert line.strip() == "ready", line
        for p in ps:
            p.stdin.write("go\n")
            p.stdin.flush()
        rc = []
        for p in ps:
            out, _ = p.communicate(timeout=max(1.0, deadline - time.time()))
            print(out.strip(), flush=True)
            rc.append(p.returncode)
    except (subprocess.TimeoutExpired, AssertionError):
        for p in ps:
            p.kill()
        for p in ps:
            p.wait()
        raise
    print("exit codes", rc, flush=True)
    sys.exit(max(rc))


if __name__ == "__main__":
    main()
