import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _unpack(bits, off, i, n):
    return np.unpackbits(bits[off[i]:off[i + 1]])[:n].astype(np.int8)


def load_encode_cases():
    """[(bg, Zc, F, ck int8[K] with -1 fillers, dn int8[N])] — reference encode_ldpc outputs."""
    d = np.load(os.path.join(GOLD, "encode_golden.npz"))
    out = []
    for i, (bg, Zc, F) in enumerate(d["meta"].tolist()):
        K = (22 if bg == 1 else 10) * Zc
        N = (66 if bg == 1 else 50) * Zc
        ck = _unpack(d["ck_bits"], d["ck_off"], i, K)
        if F:
            ck[K - F:] = -1
        par = _unpack(d["par_bits"], d["par_off"], i, N - (K - 2 * Zc))
        dn = np.concatenate([ck[2 * Zc:], par]).astype(np.int8)
        out.append((bg, Zc, F, ck, dn))
    return out


def load_decode_cases():
    """[dict(kind, bg, Zc, L, alpha, beta, llr float32[N], ck int8[Nf], status)] — reference
    nr_decode_ldpc(float64(llr), ...) outputs."""
    d = np.load(os.path.join(GOLD, "decode_golden.npz"))
    kinds = d["kinds"].tolist()
    out = []
    for i in range(d["bg"].size):
        bg, Zc = int(d["bg"][i]), int(d["Zc"][i])
        Nf = (68 if bg == 1 else 52) * Zc
        out.append(dict(kind=kinds[d["kind"][i]], bg=bg, Zc=Zc, L=int(d["L"][i]),
                        alpha=float(d["alpha"][i]), beta=float(d["beta"][i]),
                        llr=d["llr"][d["llr_off"][i]:d["llr_off"][i + 1]],
                        ck=_unpack(d["ck_bits"], d["ck_off"], i, Nf),
                        status=bool(d["status"][i])))
    return out


def load_algo_cases(algo):
    """[dict(bg, Zc, L, llr float32[N], ck int8[Nf], status)] — reference nr_decode_ldpc with
    algo='BF' / 'BP' (tests/golden/decode_{bf,bp}_golden.npz)."""
    d = np.load(os.path.join(GOLD, f"decode_{algo.lower()}_golden.npz"))
    out = []
    for i in range(d["bg"].size):
        bg, Zc = int(d["bg"][i]), int(d["Zc"][i])
        Nf = (68 if bg == 1 else 52) * Zc
        out.append(dict(bg=bg, Zc=Zc, L=int(d["L"][i]),
                        llr=d["llr"][d["llr_off"][i]:d["llr_off"][i + 1]],
                        ck=_unpack(d["ck_bits"], d["ck_off"], i, Nf), status=bool(d["status"][i])))
    return out


def load_sparse_cases():
    """[dict(kind, H uint8 (M, N), L, algo, alpha, beta, llr float32[N], ck int8[N], status)] —
    reference decode_ldpc(float64(llr), H, ...) on non-38.212 matrices
    (tests/golden/sparse_golden.npz), and the nr_decode_ldpc beta < 0 cases as a second list."""
    d = np.load(os.path.join(GOLD, "sparse_golden.npz"))
    kinds = d["kinds"].tolist()
    out = []
    for i in range(d["M"].size):
        M, N = int(d["M"][i]), int(d["N"][i])
        H = _unpack(d["H"], d["H_off"], i, M * N).astype(np.uint8).reshape(M, N)
        out.append(dict(kind=kinds[d["kind"][i]], H=H, L=int(d["L"][i]), algo=str(d["algo"][i]),
                        alpha=float(d["alpha"][i]), beta=float(d["beta"][i]),
                        llr=d["llr"][d["llr_off"][i]:d["llr_off"][i + 1]],
                        ck=_unpack(d["ck_bits"], d["ck_off"], i, N), status=bool(d["status"][i])))
    nr = []
    for i, (bg, Zc) in enumerate(d["nr_meta"].tolist()):
        Nf = (68 if bg == 1 else 52) * Zc
        nr.append(dict(bg=bg, Zc=Zc, alpha=float(d["nr_ab"][i][0]), beta=float(d["nr_ab"][i][1]),
                       llr=d["nr_llr"][d["nr_llr_off"][i]:d["nr_llr_off"][i + 1]],
                       ck=_unpack(d["nr_ck"], d["nr_ck_off"], i, Nf),
                       status=bool(d["nr_status"][i])))
    return out, nr


def load_json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def encode_cases():
    return load_encode_cases()


@pytest.fixture(scope="session")
def decode_cases():
    return load_decode_cases()
