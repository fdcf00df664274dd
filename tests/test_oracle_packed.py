"""The packed SmaQ container's restatement (oracle/smaq_packed.py) against the reference.

unpack(pack(x)) must reproduce smart.py's outputs bit for bit: checked on every golden case the
container supports (all but the BatchNorm variant), with the reference's own statistics and
recorded rand_like draws; plus escape-heavy inputs (NaN, +-inf, huge outliers, wrong-sign codes)
and ragged sizes, where it must equal oracle.smaq.apply.
"""

import numpy as np
import pytest

from helpers import load_smaq, n_diff_f32, oracle_cfg, same_f32, smaq_cases

CASES = smaq_cases()
PACKABLE = sorted(k for k, m in CASES.items() if not k.startswith("n7")
                  and not m.get("use_batch_norm") and m["main_std_dev_threshold"] > 0)


@pytest.mark.parametrize("name", PACKABLE)
def test_packed_roundtrip_matches_reference(name):
    from oracle import smaq_packed as P

    meta, d = CASES[name], load_smaq(name)
    if "bn_gamma" in d:
        pytest.skip("BatchNorm variant")
    cfg = oracle_cfg(meta)
    st = P.pack(d["x"], d["mean"], d["std"], cfg, d.get("uniforms"), meta["all_positive"],
                meta["dtype"])
    h = P.header(st)
    assert h["total_bytes"] == st.size and h["n"] == d["x"].size
    y = P.unpack(st).reshape(d["y"].shape)
    assert same_f32(y, d["y"]), n_diff_f32(y, d["y"])


@pytest.mark.parametrize("n", [1, 7, 4095, 4096, 4097, 3 * 4096 + 5])
@pytest.mark.parametrize("bits", [(6, 8), (4, 6), (2, 3), (9, 12)])
def test_packed_escapes_and_sizes(n, bits):
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from oracle import smaq_packed as P

    rs = np.random.default_rng(n * 31 + bits[0])
    x = rs.standard_t(1.5, n).astype(np.float32) * 3  # very heavy tails: many escapes
    x[rs.random(n) < 0.02] = np.nan
    x[rs.random(n) < 0.01] = np.inf
    x[rs.random(n) < 0.01] = -np.inf
    cfg = osmaq.SmaqConfig(num_bits_main=bits[0], num_bits_outlier=bits[1])
    u = orng.uniforms(3, 5, n)
    mean, std = np.float32(0.25), np.float32(1.5)
    st = P.pack(x, mean, std, cfg, u)
    y_ref, _ = osmaq.apply(x, mean, std, cfg, u)
    assert same_f32(P.unpack(st), y_ref)
    for all_pos in (True,):
        st = P.pack(x, mean, std, cfg, u, all_positive=all_pos)
        y_ref, _ = osmaq.apply(x, mean, std, cfg, u, all_positive=all_pos)
        assert same_f32(P.unpack(st), y_ref)


def test_code_stream_layout():
    """Codes in element order, LSB-first, width wm (main) or wo (outlier): element e at bit
    wm * e + (wo - wm) * (outliers before e)."""
    from oracle import smaq_packed as P

    cb = np.array([1, 0x45, 2, 3], np.uint64)
    ob = np.array([False, True, False, False])
    w = P._code_stream(cb, ob, 5, 7)
    assert w.size == 1 and w[0] == (1 | (0x45 << 5) | (2 << 12) | (3 << 17))
    rs = np.random.default_rng(0)
    for wm, wo in ((5, 7), (1, 2), (13, 24)):
        ob = rs.random(1000) < 0.3
        cb = np.where(ob, rs.integers(0, 2**wo, 1000), rs.integers(0, 2**wm, 1000)).astype(np.uint64)
        words = P._code_stream(cb, ob, wm, wo)
        assert words.size == (wm * 1000 + (wo - wm) * int(ob.sum()) + 31) // 32
