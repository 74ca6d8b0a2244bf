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


def load_json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def encode_cases():
    return load_encode_cases()


@pytest.fixture(scope="session")
def decode_cases():
    return load_decode_cases()
