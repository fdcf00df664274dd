"""The packed SmaQ container's restatement (oracle/smaq_packed.py) against the reference.

unpack(pack(x)) must reproduce smart.py's outputs bit for bit: checked on every golden case (the
BatchNorm variant and negative thresholds included), with the reference's own statistics and
recorded rand_like draws; plus escape-heavy inputs (NaN, +-inf, huge outliers, wrong-sign codes)
and ragged sizes, where it must equal oracle.smaq.apply.
"""

import numpy as np
import pytest

from helpers import load_smaq, n_diff_f32, oracle_cfg, same_f32, smaq_cases

CASES = smaq_cases()
PACKABLE = sorted(k for k in CASES if not k.startswith("n7"))  # (n7: below min_size, kept raw)


@pytest.mark.parametrize("name", PACKABLE)
def test_packed_roundtrip_matches_reference(name):
    from oracle import smaq_packed as P

    meta, d = CASES[name], load_smaq(name)
    bn = None
    if "bn_gamma" in d:
        bn = (d["bn_gamma_used"], d["bn_beta_used"]) if meta["bn_scalar_params"] else (
            d["bn_gamma"], d["bn_beta"])
    cfg = oracle_cfg(meta)
    st = P.pack(d["x"], d["mean"], d["std"], cfg, d.get("uniforms"), meta["all_positive"],
                meta["dtype"], bn)
    h = P.header(st)
    assert h["total_bytes"] == st.size and h["n"] == d["x"].size
    assert bool(h["flags"] & P.FLAG_BN) == (bn is not None)
    assert bool(h["flags"] & P.FLAG_BOTH_SIDES) == (meta["main_std_dev_threshold"] < 0)
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


def test_fixed_and_variable_layout():
    """Format v2: a block's fixed section is 128 mask words + the plane (the low wm bits of every
    code at bit wm * e); its variable section holds the outliers' remaining wo - wm code bits in
    element order, then the escapes. Each block's fixed section sits at b * F words (no prefix
    needed to place it), the directory locates the variable sections."""
    from oracle import smaq_packed as P

    cb = np.array([1, 0x45, 2, 3], np.uint64)
    ob = np.array([False, True, False, False])
    fx = P.block_fixed(cb, ob, 5)
    assert fx.size == P.fixed_words(5) == 128 + 5 * 128
    assert fx[0] == 0b0010 and not fx[1:128].any()
    assert fx[128] == (1 | ((0x45 & 31) << 5) | (2 << 10) | (3 << 15)) and not fx[129:].any()
    v = P.block_var(cb, ob, np.zeros(4, bool), np.zeros(4, np.float32), 5, 7)
    assert v.size == 1 and v[0] == (0x45 >> 5)
    rs = np.random.default_rng(0)
    for wm, wo in ((5, 7), (1, 2), (13, 24), (6, 4)):
        ob = rs.random(1000) < 0.3
        cb = np.where(ob, rs.integers(0, 2**wo, 1000), rs.integers(0, 2**wm, 1000)).astype(np.uint64)
        eb = rs.random(1000) < 0.01
        v = P.block_var(cb, ob, eb, rs.standard_normal(1000).astype(np.float32), wm, wo)
        assert v.size == (max(0, wo - wm) * int(ob.sum()) + 31) // 32 + 2 * int(eb.sum())
    x = rs.standard_normal(3 * 4096 + 5).astype(np.float32) * 3
    from oracle import smaq as osmaq

    st = P.pack(x, np.float32(0.1), np.float32(2.0), osmaq.SmaqConfig(stochastic_rounding=False))
    h, dirs, fixed_w, var_w = P.regions(st)
    assert fixed_w.size == 4 * P.fixed_words(5) and h["data_words"] == var_w.size
    off = (dirs & np.uint64((1 << 38) - 1)).astype(np.int64)
    n_out = ((dirs >> np.uint64(38)) & np.uint64(0x1FFF)).astype(np.int64)
    n_esc = (dirs >> np.uint64(51)).astype(np.int64)
    size = (2 * n_out + 31) // 32 + 2 * n_esc
    assert off[0] == 0 and np.array_equal(np.diff(off), size[:-1]) and off[-1] + size[-1] == var_w.size
