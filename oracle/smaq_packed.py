"""TEST INFRASTRUCTURE ONLY — numpy restatement of the packed SmaQ container (include/smq.h,
"Packed SmaQ container", format version 2). The product never imports this module.

What it pins: the codes are smart.py's own (oracle.smaq.codes, smart.py:144-169); the container
stores them losslessly (escape list for anything outside the [outlier flag][sign][N-2 magnitude]
budget of README.md:25-28), so ``unpack(pack(x))`` must equal ``oracle.smaq.apply`` — which is
pinned bit-for-bit to the reference by the golden vectors. The byte layout itself is this
repository's (the reference has no packed container in smart.py; its HLS layout in hw/smaq.cpp
needs Xilinx headers and is not built here), so the GPU stream is compared byte for byte with
this restatement.
"""

import struct
from typing import Optional

import numpy as np

from . import smaq as osmaq

F32 = np.float32
MAGIC = 0x50514D53
VERSION = 2
BLOCK = 4096
HEADER_BYTES = 128
MASK_WORDS = BLOCK // 32
_HDR = struct.Struct("<IIqIIiiIfffffddQQIIqdd8x")
FLAG_BOTH_SIDES = 4
FLAG_BN = 8
FLAG_F64 = 16
NAN64 = 0x7FF8000000000000
assert _HDR.size == HEADER_BYTES


def _widths(bm: int, bo: int):
    return bm - 1, bo - 1


def fixed_words(wm: int) -> int:
    """Words of a block's fixed section: the outlier mask, then the plane of wm bits per element."""
    return MASK_WORDS + (wm * BLOCK) // 32


def _flags(all_positive: bool, r_main: np.float32, r_out: np.float32, thr=1.0, bn=False) -> int:
    lim = 2.0**100
    safe_q = not (abs(float(r_main)) <= lim and abs(float(r_out)) <= lim)  # smaq_elem.h RangeRecips
    return ((1 if all_positive else 0) | (2 if safe_q else 0) |
            (FLAG_BOTH_SIDES if F32(thr) < 0 else 0) | (FLAG_BN if bn else 0))


def block_codes(q, hi, lo, wm: int, wo: int):
    """Per element: (code, mask bit, escaped) — smq.h packed format rules. The mask bit is "exactly
    one side" (T < 0 also gives elements with both sides: they code as main elements). A main code
    is the wm-bit two's complement q; an outlier code is side << (wo - 1) | |q| (wo bits); a code
    outside the budget is 0 (main) or the side bit alone (outlier) and the element is escaped."""
    o = hi ^ lo
    hi, lo = hi & o, lo & o
    with np.errstate(invalid="ignore"):
        main_lo, main_hi = -(2 ** (wm - 1)), 2 ** (wm - 1) - 1
        mag_max = 2 ** (wo - 1) - 1
        ok_main = (q >= main_lo) & (q <= main_hi)
        ok_hi = (q >= 0) & (q <= mag_max)
        ok_lo = (q <= 0) & (-q <= mag_max)
    ok = np.where(o, np.where(hi, ok_hi, ok_lo), ok_main)
    qi = np.where(ok, q, 0).astype(np.int64)
    main_code = qi & ((1 << wm) - 1)
    side = lo.astype(np.int64) << (wo - 1)
    out_code = side | np.where(hi, qi, -qi)
    code = np.where(o, np.where(ok, out_code, side), np.where(ok, main_code, 0))
    return code.astype(np.uint64), o, ~ok


def _pack_bits(codes: np.ndarray, width: int) -> np.ndarray:
    """LSB-first concatenation of ``width``-bit codes into uint32 words."""
    n = codes.size
    words = (width * n + 31) // 32
    if n == 0 or width == 0:
        return np.zeros(0, np.uint32)
    bits = ((codes[:, None] >> np.arange(width, dtype=np.uint64)) & 1).astype(np.uint8).ravel()
    bits = np.concatenate([bits, np.zeros(words * 32 - bits.size, np.uint8)])
    return np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32)


def _unpack_bits(words: np.ndarray, width: int, n: int) -> np.ndarray:
    if n == 0 or width == 0:
        return np.zeros(n, np.uint64)
    bits = np.unpackbits(np.asarray(words, np.uint32).astype(">u4").view(np.uint8).reshape(-1, 4),
                         axis=1)
    bits = bits.reshape(-1, 32)[:, ::-1].ravel()[: width * n].reshape(n, width).astype(np.uint64)
    return (bits << np.arange(width, dtype=np.uint64)).sum(axis=1)


def block_fixed(cb, ob, wm: int) -> np.ndarray:
    """The fixed section of one block: 128 mask words (bit e % 32 of word e // 32: element e is an
    outlier), then the plane: the low wm bits of every element's code at bit wm * e (absent
    elements of a short last block are zero)."""
    m = cb.size
    mask = np.zeros(BLOCK, np.uint8)
    mask[:m] = ob
    mask_words = np.packbits(mask.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel()
    plane = np.zeros(BLOCK, np.uint64)
    plane[:m] = cb & np.uint64((1 << wm) - 1)
    return np.concatenate([mask_words.astype(np.uint32), _pack_bits(plane, wm)])


def block_var(cb, ob, eb, qb, wm: int, wo: int) -> np.ndarray:
    """The variable section of one block: the outliers' code bits above the plane (we = wo - wm
    bits each, in element order, LSB-first; none when wo <= wm), then the escapes {element index
    in the block, q as float32 bits} in element order."""
    we = max(0, wo - wm)
    ext = _pack_bits(cb[ob] >> np.uint64(wm), we)
    esc_idx = np.nonzero(eb)[0].astype(np.uint32)
    qe = np.asarray(qb, F32)[esc_idx]
    qbits = np.where(np.isnan(qe), np.uint32(0x7FC00000), qe.view(np.uint32))  # one NaN pattern
    esc_words = np.stack([esc_idx, qbits.astype(np.uint32)], axis=1).ravel()
    return np.concatenate([ext, esc_words.astype(np.uint32)])


def pack_block(xb, mean, std, cfg: osmaq.SmaqConfig, uniforms=None, dtype: str = "f32"):
    """(fixed, variable) sections of one block's elements (no BN)."""
    wm, wo = _widths(cfg.num_bits_main, cfg.num_bits_outlier)
    q, hi, lo, _ = osmaq.codes(np.asarray(xb, F32).ravel(), mean, std, cfg, uniforms, None, dtype)
    code, o, esc = block_codes(q, hi, lo, wm, wo)
    return block_fixed(code, o, wm), block_var(code, o, esc, q, wm, wo)


def pack(x, mean, std, cfg: osmaq.SmaqConfig, uniforms: Optional[np.ndarray] = None,
         all_positive: bool = False, dtype: str = "f32", bn=None) -> np.ndarray:
    """The stream smq_smaq_compress writes, given the device statistics (mean, raw std) and the
    same uniforms. Returns uint8 bytes: header | directory (padded to an even number of entries)
    | fixed region | variable region [| BN table] — every region's place but the variable one's
    depends on n alone, and the fixed region is 16-B aligned. bn = (gamma, beta) of the channels
    of dim 1 (x NCHW; one value each for scalar parameters)."""
    x = np.asarray(x, dtype=F32)
    inner = 0
    if bn is not None:
        assert x.ndim == 4
        inner = x.shape[2] * x.shape[3]
        bn = tuple(np.asarray(t, F32).reshape(-1) for t in bn)
    q, hi, lo, std1 = osmaq.codes(x, mean, std, cfg, uniforms, bn, dtype)
    q, hi, lo = q.ravel(), hi.ravel(), lo.ravel()
    x = x.ravel()
    n = x.size
    bm, bo = cfg.num_bits_main, cfg.num_bits_outlier
    wm, wo = _widths(bm, bo)
    code, o, esc = block_codes(q, hi, lo, wm, wo)
    nb = (n + BLOCK - 1) // BLOCK
    fixed, var, dirs, off = [], [], [], 0
    for b in range(nb):
        s = slice(b * BLOCK, min(n, (b + 1) * BLOCK))
        fixed.append(block_fixed(code[s], o[s], wm))
        v = block_var(code[s], o[s], esc[s], q[s], wm, wo)
        # directory entry: variable-section word offset (38 bits) | n_out << 38 | n_esc << 51
        dirs.append(off | (int(o[s].sum()) << 38) | (int(esc[s].sum()) << 51))
        off += v.size
        var.append(v)
    fixed_w = np.concatenate(fixed) if fixed else np.zeros(0, np.uint32)
    var_w = np.concatenate(var) if var else np.zeros(0, np.uint32)
    r_main, r_out = F32(cfg.range_normal), F32(cfg.range_outlier)
    nbp = nb + (nb & 1)
    bn_tab = np.concatenate([bn[0], bn[1]]).astype(F32) if bn is not None else np.zeros(0, F32)
    total = HEADER_BYTES + 8 * nbp + 4 * (fixed_w.size + var_w.size + bn_tab.size)
    thr = F32(cfg.main_std_dev_threshold)
    hdr = _HDR.pack(MAGIC, VERSION, n, BLOCK, nb, bm, bo,
                    _flags(all_positive, r_main, r_out, thr, bn is not None),
                    thr, r_main, r_out, F32(mean), F32(std1),
                    1.0 / float(r_main) if r_main != 0 else float("inf"),
                    1.0 / float(r_out) if r_out != 0 else float("inf"),
                    var_w.size, total, 0, bn_tab.size // 2, inner, 0.0, 0.0)
    dirs += [0] * (nbp - nb)
    return np.concatenate([np.frombuffer(hdr, np.uint8), np.asarray(dirs, np.uint64).view(np.uint8),
                           fixed_w.view(np.uint8), var_w.view(np.uint8), bn_tab.view(np.uint8)])


def header(stream: np.ndarray) -> dict:
    f = _HDR.unpack(bytes(np.asarray(stream[:HEADER_BYTES], np.uint8)))
    keys = ("magic", "version", "n", "block_elems", "n_blocks", "num_bits_main",
            "num_bits_outlier", "flags", "thr", "range_main", "range_outlier", "mean", "std_dev",
            "inv_range_main", "inv_range_outlier", "data_words", "total_bytes", "error",
            "bn_channels", "bn_inner", "mean_f64", "std_dev_f64")
    return dict(zip(keys, f))


def regions(stream: np.ndarray):
    """(header dict, directory uint64[nb], fixed region uint32[nb * F], variable region uint32
    (without a BN stream's table: bn_table())."""
    h = header(stream)
    nb = h["n_blocks"]
    wm = h["num_bits_main"] - 1
    nbp = nb + (nb & 1)
    dirs = np.asarray(stream[HEADER_BYTES: HEADER_BYTES + 8 * nb], np.uint8).view(np.uint64)
    f0 = HEADER_BYTES + 8 * nbp
    fb = 4 * nb * fixed_words(wm)
    fixed_w = np.asarray(stream[f0: f0 + fb], np.uint8).view(np.uint32)
    var_w = np.asarray(stream[f0 + fb: f0 + fb + 4 * h["data_words"]], np.uint8).view(np.uint32)
    return h, dirs, fixed_w, var_w


def bn_table(stream: np.ndarray):
    """A BN stream's (gamma, beta) (fp32, bn_channels each), after the variable region."""
    h = header(stream)
    nb = h["n_blocks"]
    off = (HEADER_BYTES + 8 * (nb + (nb & 1)) + 4 * nb * fixed_words(h["num_bits_main"] - 1)
           + 4 * h["data_words"])
    c = h["bn_channels"]
    t = np.asarray(stream[off: off + 8 * c], np.uint8).view(F32)
    return t[:c], t[c:]


def block_var_f64(cb, ob, eb, qb, wm: int, wo: int) -> np.ndarray:
    """A float64 stream's variable section: the outlier bits above the plane, then the escapes
    {element index, q as float64 bits low word, high word} (any NaN q as 0x7ff8000000000000)."""
    we = max(0, wo - wm)
    ext = _pack_bits(cb[ob] >> np.uint64(wm), we)
    esc_idx = np.nonzero(eb)[0].astype(np.uint32)
    qe = np.asarray(qb, np.float64)[esc_idx]
    qbits = np.where(np.isnan(qe), np.uint64(NAN64), qe.view(np.uint64))
    esc = np.stack([esc_idx, (qbits & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                    (qbits >> np.uint64(32)).astype(np.uint32)], axis=1).ravel()
    return np.concatenate([ext, esc.astype(np.uint32)])


def pack_f64(x, mean, std, cfg: osmaq.SmaqConfig, uniforms: Optional[np.ndarray] = None,
             all_positive: bool = False, bn=None) -> np.ndarray:
    """The float64 stream smq_smaq_compress_f64 writes (flag FLAG_F64), given the device's fp64
    statistics (mean, raw std) and the same uniforms: the codes of osmaq.codes_f64 (smart.py on a
    float64 tensor), 3-word escapes, the statistics (std after the ==0 rule) as doubles, an fp64
    BN table."""
    x = np.asarray(x, dtype=np.float64)
    inner = 0
    if bn is not None:
        assert x.ndim == 4
        inner = x.shape[2] * x.shape[3]
        bn = tuple(np.asarray(t, np.float64).reshape(-1) for t in bn)
    q, hi, lo = osmaq.codes_f64(x, mean, std, cfg, uniforms, bn)
    q, hi, lo = q.ravel(), hi.ravel(), lo.ravel()
    n = x.size
    bm, bo = cfg.num_bits_main, cfg.num_bits_outlier
    wm, wo = _widths(bm, bo)
    code, o, esc = block_codes(q, hi, lo, wm, wo)
    nb = (n + BLOCK - 1) // BLOCK
    fixed, var, dirs, off = [], [], [], 0
    for b in range(nb):
        s = slice(b * BLOCK, min(n, (b + 1) * BLOCK))
        fixed.append(block_fixed(code[s], o[s], wm))
        v = block_var_f64(code[s], o[s], esc[s], q[s], wm, wo)
        dirs.append(off | (int(o[s].sum()) << 38) | (int(esc[s].sum()) << 51))
        off += v.size
        var.append(v)
    fixed_w = np.concatenate(fixed) if fixed else np.zeros(0, np.uint32)
    var_w = np.concatenate(var) if var else np.zeros(0, np.uint32)
    r_main, r_out = F32(cfg.range_normal), F32(cfg.range_outlier)
    nbp = nb + (nb & 1)
    bn_tab = (np.concatenate([bn[0], bn[1]]).astype(np.float64) if bn is not None
              else np.zeros(0, np.float64))
    total = HEADER_BYTES + 8 * nbp + 4 * (fixed_w.size + var_w.size) + 8 * bn_tab.size
    thr = F32(cfg.main_std_dev_threshold)
    std1 = np.float64(std) if np.float64(std) != 0 else np.float64(1.0)
    hdr = _HDR.pack(MAGIC, VERSION, n, BLOCK, nb, bm, bo,
                    FLAG_F64 | _flags(all_positive, r_main, r_out, thr, bn is not None),
                    thr, r_main, r_out, F32(mean), F32(std1),
                    1.0 / float(r_main) if r_main != 0 else float("inf"),
                    1.0 / float(r_out) if r_out != 0 else float("inf"),
                    var_w.size, total, 0, bn_tab.size // 2, inner, float(mean), float(std1))
    dirs += [0] * (nbp - nb)
    return np.concatenate([np.frombuffer(hdr, np.uint8), np.asarray(dirs, np.uint64).view(np.uint8),
                           fixed_w.view(np.uint8), var_w.view(np.uint8), bn_tab.view(np.uint8)])


def unpack(stream: np.ndarray) -> np.ndarray:
    """Decode a stream (smq_smaq_decompress[_f64]): fp32 values in element order (float64 for a
    float64 stream)."""
    h, dirs, fixed_w, var_w = regions(stream)
    assert h["magic"] == MAGIC and h["version"] == VERSION
    f64 = bool(h["flags"] & FLAG_F64)
    ew = 3 if f64 else 2
    n, nb = h["n"], h["n_blocks"]
    wm, wo = _widths(h["num_bits_main"], h["num_bits_outlier"])
    we = max(0, wo - wm)
    F = fixed_words(wm)
    q = np.zeros(n, np.float64 if f64 else F32)
    hi = np.zeros(n, bool)
    lo = np.zeros(n, bool)
    for b in range(nb):
        m = min(BLOCK, n - b * BLOCK)
        d = int(dirs[b])
        base, n_out, n_esc = d & ((1 << 38) - 1), (d >> 38) & 0x1FFF, d >> 51
        fx = fixed_w[b * F: (b + 1) * F]
        mask_bits = np.unpackbits(fx[:MASK_WORDS].astype(">u4").view(np.uint8)
                                  .reshape(-1, 4), axis=1).reshape(-1, 32)[:, ::-1].ravel()
        ob = mask_bits[:m].astype(bool)
        assert int(ob.sum()) == n_out
        cd = _unpack_bits(fx[MASK_WORDS:], wm, m)
        n_ext = (we * n_out + 31) // 32
        ext = _unpack_bits(var_w[base: base + n_ext], we, n_out)
        cd[ob] |= ext << np.uint64(wm)
        cd = cd.astype(np.int64)
        qm = np.where(cd >= 2 ** (wm - 1), cd - 2**wm, cd)
        side = (cd >> (wo - 1)) & 1
        mag = cd & ((1 << (wo - 1)) - 1)
        qo = np.where(side == 1, -mag, mag)
        qb = np.where(ob, qo, qm).astype(np.float64 if f64 else F32)
        both = bool(h["flags"] & FLAG_BOTH_SIDES)  # a mask-0 element has both sides
        hb = np.where(ob, side == 0, both)
        lb = np.where(ob, side == 1, both)
        e = var_w[base + n_ext: base + n_ext + ew * n_esc].reshape(-1, ew)
        if f64:
            qb[e[:, 0].astype(np.int64)] = (e[:, 1].astype(np.uint64)
                                            | (e[:, 2].astype(np.uint64) << np.uint64(32))
                                            ).view(np.float64)
        else:
            qb[e[:, 0].astype(np.int64)] = e[:, 1].view(F32)
        s = slice(b * BLOCK, b * BLOCK + m)
        q[s], hi[s], lo[s] = qb, hb, lb
    if f64:
        bn, ch = None, None
        if h["flags"] & FLAG_BN:
            nbp = nb + (nb & 1)
            off = (HEADER_BYTES + 8 * nbp + 4 * nb * fixed_words(wm) + 4 * h["data_words"])
            c = h["bn_channels"]
            t = np.asarray(stream[off: off + 16 * c], np.uint8).view(np.float64)
            bn = (t[:c], t[c:])
            ch = (np.arange(n, dtype=np.int64) // h["bn_inner"]) % c
        return osmaq.dequant_f64(q, hi, lo, h["mean_f64"], h["std_dev_f64"], h["thr"],
                                 h["range_main"], h["range_outlier"], bool(h["flags"] & 1), bn, ch)
    cfg = osmaq.SmaqConfig(num_bits_main=h["num_bits_main"], num_bits_outlier=h["num_bits_outlier"],
                           main_std_dev_threshold=float(F32(h["thr"])))
    # the ranges come from the header (the compressor's fp32 constants)
    cfg_r = _RangesCfg(cfg, F32(h["range_main"]), F32(h["range_outlier"]))
    if h["flags"] & FLAG_BN:  # per element: channel (e / inner) % channels (NCHW dim 1)
        g, b = bn_table(stream)
        ch = (np.arange(n, dtype=np.int64) // h["bn_inner"]) % h["bn_channels"]
        y = osmaq.dequant(q, hi, lo, h["mean"], h["std_dev"], cfg_r, False)
        with np.errstate(all="ignore"):
            y = (y * g[ch]) + b[ch]
            if h["flags"] & 1:
                y = np.where(y < F32(0), F32(0), y)
        return y.astype(F32)
    return osmaq.dequant(q, hi, lo, h["mean"], h["std_dev"], cfg_r, bool(h["flags"] & 1))


class _RangesCfg:
    """A SmaqConfig view with explicit fp32 ranges (those recorded in the stream header)."""

    def __init__(self, cfg, r_main, r_out):
        self._cfg = cfg
        self.range_normal = r_main
        self.range_outlier = r_out

    def __getattr__(self, k):
        return getattr(self._cfg, k)
