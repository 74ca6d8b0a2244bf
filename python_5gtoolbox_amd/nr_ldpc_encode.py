"""Drop-in for py5gphy/ldpc/nr_ldpc_encode.py, backed by the HIP encoder (ldpc5g_encode).

    encode_ldpc(ck, bgn) -> dn                    (reference: nr_ldpc_encode.py:8-50)
    encode_ldpc_batch(cbs, bgn) -> dn[B, N]       (batched; numpy or device tensors)

Reference semantics kept: AssertionError on a bad bgn / lifting size; dn is int8 of length
N = 66Zc (BG1) / 50Zc (BG2) with dn[0:K-2Zc] = ck[2Zc:K] (fillers stay -1) and the parity
after; filler entries (-1) of the caller's ck at k >= 2Zc are zeroed IN PLACE
(nr_ldpc_encode.py:32-37).  There is no CPU fallback.
"""
import numpy as np

from . import _lib
from .ldpc_info import find_iLS


def _dims(K, bgn):
    if bgn == 1:
        Zc = K // 22
        return Zc, 66 * Zc
    Zc = K // 10
    return Zc, 50 * Zc


def encode_ldpc_batch(cbs, bgn, out=None):
    """Encode B codeblocks at once.

    cbs: (B, K) int8 array — numpy (copied to the GPU and back) or a torch tensor on the GPU
    (stays there; `out` may supply a preallocated (B, >=N) int8 device tensor).
    Returns dn (B, N) of the same kind.  The input is not modified."""
    assert bgn in [1, 2]
    t = _lib.require_gpu()
    is_np = not isinstance(cbs, t.Tensor)
    x = t.from_numpy(np.ascontiguousarray(cbs, dtype=np.int8)) if is_np else cbs
    assert x.dim() == 2 and x.dtype == t.int8
    B, K = x.shape
    Zc, N = _dims(K, bgn)
    assert find_iLS(Zc) < 8 and K == (22 if bgn == 1 else 10) * Zc, f"bad codeblock size K={K}"
    if is_np:
        x = x.cuda()
    if x.stride(1) != 1:
        x = x.contiguous()
    if out is None:
        out = t.empty((B, N), dtype=t.int8, device=x.device)
    assert out.dtype == t.int8 and out.shape[0] == B and out.shape[1] >= N and out.stride(1) == 1
    with t.cuda.device(x.device):
        _lib.check(_lib.lib().ldpc5g_encode(_lib.ptr(x), _lib.ptr(out), B, bgn, Zc, x.stride(0),
                                            out.stride(0), _lib.stream_ptr(x.device)))
    if is_np:
        return out[:, :N].cpu().numpy()
    return out


def encode_ldpc(ck, bgn):
    """LDPC encode following TS 38.212 5.3.2 — drop-in for nr_ldpc_encode.encode_ldpc.

    input:  ck: K length code block (values 0/1, -1 = filler), bgn: base graph 1 or 2
    output: dn: N length LDPC encoded sequence (int8)"""
    assert bgn in [1, 2]
    K = ck.size
    Zc, N = _dims(K, bgn)
    iLS = find_iLS(Zc)
    assert iLS < 8
    _lib.require_gpu()
    # host rows straight through the library (ldpc5g_encode_host: its per-thread pinned / device
    # staging, one H2D, the launch, one D2H, one synchronisation — no torch op on the way)
    x = np.ascontiguousarray(np.asarray(ck).reshape(-1), dtype=np.int8)
    dn = np.empty(N, np.int8)
    _lib.check(_lib.lib().ldpc5g_encode_host(x.ctypes.data, dn.ctypes.data, 1, bgn, Zc,
                                             _lib.stream_ptr()))
    # reference side effect: fillers of the caller's block are zeroed in place (:34-35)
    tail = ck[2 * Zc:K]
    tail[tail == -1] = 0
    return dn
