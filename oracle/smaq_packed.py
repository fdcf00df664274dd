"""TEST INFRASTRUCTURE ONLY — numpy restatement of the packed SmaQ container (include/smq.h,
"Packed SmaQ container", format version 1). The product never imports this module.

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
VERSION = 1
BLOCK = 4096
HEADER_BYTES = 128
_HDR = struct.Struct("<IIqIIiiIfffffddQQI36x")
assert _HDR.size == HEADER_BYTES


def _widths(bm: int, bo: int):
    return bm - 1, bo - 1


def _flags(all_positive: bool, r_main: np.float32, r_out: np.float32) -> int:
    lim = 2.0**100
    safe_q = not (abs(float(r_main)) <= lim and abs(float(r_out)) <= lim)  # smaq_elem.h RangeRecips
    return (1 if all_positive else 0) | (2 if safe_q else 0)


def block_codes(q, hi, lo, wm: int, wo: int):
    """Per element: (plane code, is_outlier, escaped) — smq.h packed format rules."""
    o = hi | lo
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
    if n == 0:
        return np.zeros(0, np.uint32)
    bits = ((codes[:, None] >> np.arange(width, dtype=np.uint64)) & 1).astype(np.uint8).ravel()
    bits = np.concatenate([bits, np.zeros(words * 32 - bits.size, np.uint8)])
    return np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32)


def _unpack_bits(words: np.ndarray, width: int, n: int) -> np.ndarray:
    if n == 0:
        return np.zeros(0, np.uint64)
    bits = np.unpackbits(words.astype(">u4").view(np.uint8).reshape(-1, 4), axis=1)
    bits = bits.reshape(-1, 32)[:, ::-1].ravel()[: width * n].reshape(n, width).astype(np.uint64)
    return (bits << np.arange(width, dtype=np.uint64)).sum(axis=1)


def _code_stream(cb, ob, wm: int, wo: int) -> np.ndarray:
    """Codes concatenated LSB-first in ELEMENT order: element e's code (wm bits if main, wo bits if
    outlier) starts at bit wm * e + (wo - wm) * (outliers before e)."""
    widths = np.where(ob, wo, wm).astype(np.int64)
    n = cb.size
    total = int(widths.sum())
    words = (total + 31) // 32
    if n == 0:
        return np.zeros(0, np.uint32)
    wmax = max(wm, wo)
    bits = ((cb[:, None] >> np.arange(wmax, dtype=np.uint64)) & 1).astype(np.uint8)
    keep = np.arange(wmax)[None, :] < widths[:, None]
    flat = bits[keep]  # row-major: element order, LSB first within each code
    flat = np.concatenate([flat, np.zeros(words * 32 - flat.size, np.uint8)])
    return np.packbits(flat.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32)


def block_words(cb, ob, eb, qb, wm: int, wo: int) -> np.ndarray:
    """The uint32 image of one block (w[0], mask, code stream, escapes)."""
    n_out, n_esc = int(ob.sum()), int(eb.sum())
    mask = np.zeros(BLOCK, np.uint8)
    mask[: ob.size] = ob
    mask_words = np.packbits(mask.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel()
    esc_idx = np.nonzero(eb)[0].astype(np.uint32)
    esc_words = np.stack([esc_idx, qb[esc_idx].view(np.uint32)], axis=1).ravel()
    return np.concatenate([np.array([n_out | (n_esc << 16)], np.uint32),
                           mask_words.astype(np.uint32), _code_stream(cb, ob, wm, wo),
                           esc_words.astype(np.uint32)])


def pack_block(xb, mean, std, cfg: osmaq.SmaqConfig, uniforms=None, dtype: str = "f32"):
    """Image of one block's elements (the GPU stream holds it at its directory offset)."""
    wm, wo = _widths(cfg.num_bits_main, cfg.num_bits_outlier)
    q, hi, lo, _ = osmaq.codes(np.asarray(xb, F32).ravel(), mean, std, cfg, uniforms, None, dtype)
    code, o, esc = block_codes(q, hi, lo, wm, wo)
    return block_words(code, o, esc, q, wm, wo)


def pack(x, mean, std, cfg: osmaq.SmaqConfig, uniforms: Optional[np.ndarray] = None,
         all_positive: bool = False, dtype: str = "f32") -> np.ndarray:
    """The stream smq_smaq_compress writes, given the device statistics (mean, raw std) and the
    same uniforms. Returns uint8 bytes."""
    x = np.asarray(x, dtype=F32).ravel()
    n = x.size
    bm, bo = cfg.num_bits_main, cfg.num_bits_outlier
    wm, wo = _widths(bm, bo)
    q, hi, lo, std1 = osmaq.codes(x, mean, std, cfg, uniforms, None, dtype)
    code, o, esc = block_codes(q, hi, lo, wm, wo)
    nb = (n + BLOCK - 1) // BLOCK
    blocks, offsets, off = [], [], 0
    for b in range(nb):
        s = slice(b * BLOCK, min(n, (b + 1) * BLOCK))
        words = block_words(code[s], o[s], esc[s], q[s], wm, wo)
        offsets.append(off)
        off += words.size
        blocks.append(words)
    data = np.concatenate(blocks) if blocks else np.zeros(0, np.uint32)
    # directory entry: word offset (38 bits) | n_out << 38 | n_esc << 51
    counts = np.array([(int(w[0]) & 0xFFFF, int(w[0]) >> 16) for w in blocks], np.uint64).reshape(-1, 2)
    offsets = (np.asarray(offsets, np.uint64) | (counts[:, 0] << np.uint64(38))
               | (counts[:, 1] << np.uint64(51)))
    r_main, r_out = F32(cfg.range_normal), F32(cfg.range_outlier)
    total = HEADER_BYTES + 8 * nb + 4 * data.size
    hdr = _HDR.pack(MAGIC, VERSION, n, BLOCK, nb, bm, bo, _flags(all_positive, r_main, r_out),
                    F32(cfg.main_std_dev_threshold), r_main, r_out, F32(mean), F32(std1),
                    1.0 / float(r_main) if r_main != 0 else float("inf"),
                    1.0 / float(r_out) if r_out != 0 else float("inf"),
                    data.size, total, 0)
    return np.concatenate([np.frombuffer(hdr, np.uint8),
                           np.asarray(offsets, np.uint64).view(np.uint8),
                           data.view(np.uint8)])


def header(stream: np.ndarray) -> dict:
    f = _HDR.unpack(bytes(np.asarray(stream[:HEADER_BYTES], np.uint8)))
    keys = ("magic", "version", "n", "block_elems", "n_blocks", "num_bits_main",
            "num_bits_outlier", "flags", "thr", "range_main", "range_outlier", "mean", "std_dev",
            "inv_range_main", "inv_range_outlier", "data_words", "total_bytes", "error")
    return dict(zip(keys, f))


def unpack(stream: np.ndarray) -> np.ndarray:
    """Decode a stream (smq_smaq_decompress): fp32 values in element order."""
    h = header(stream)
    assert h["magic"] == MAGIC and h["version"] == VERSION
    n, nb = h["n"], h["n_blocks"]
    wm, wo = _widths(h["num_bits_main"], h["num_bits_outlier"])
    dirs = np.asarray(stream[HEADER_BYTES: HEADER_BYTES + 8 * nb], np.uint8).view(np.uint64)
    dirs = dirs & np.uint64((1 << 38) - 1)  # word offsets (n_out / n_esc also live in w[0])
    data = np.asarray(stream[HEADER_BYTES + 8 * nb:], np.uint8).view(np.uint32)
    q = np.zeros(n, F32)
    hi = np.zeros(n, bool)
    lo = np.zeros(n, bool)
    for b in range(nb):
        base = int(dirs[b])
        m = min(BLOCK, n - b * BLOCK)
        w0 = int(data[base])
        n_out, n_esc = w0 & 0xFFFF, w0 >> 16
        mask_bits = np.unpackbits(data[base + 1: base + 129].astype(">u4").view(np.uint8)
                                  .reshape(-1, 4), axis=1).reshape(-1, 32)[:, ::-1].ravel()
        ob = mask_bits[:m].astype(bool)
        p = base + 129
        nw = (wm * m + (wo - wm) * n_out + 31) // 32
        bits = np.unpackbits(data[p: p + nw].astype(">u4").view(np.uint8).reshape(-1, 4),
                             axis=1).reshape(-1, 32)[:, ::-1].ravel().astype(np.uint64)
        r_out = np.concatenate([[0], np.cumsum(ob)[:-1]]).astype(np.int64)
        pos = wm * np.arange(m, dtype=np.int64) + (wo - wm) * r_out
        widths = np.where(ob, wo, wm)
        cd = np.zeros(m, np.uint64)
        for t in range(max(wm, wo)):
            sel = t < widths
            cd[sel] |= bits[pos[sel] + t] << np.uint64(t)
        cd = cd.astype(np.int64)
        qm = np.where(cd >= 2 ** (wm - 1), cd - 2**wm, cd)
        side = (cd >> (wo - 1)) & 1
        mag = cd & ((1 << (wo - 1)) - 1)
        qo = np.where(side == 1, -mag, mag)
        qb = np.where(ob, qo, qm).astype(F32)
        hb = ob & (side == 0)
        lb = ob & (side == 1)
        e = data[p + nw: p + nw + 2 * n_esc].reshape(-1, 2)
        qb[e[:, 0].astype(np.int64)] = e[:, 1].view(F32)
        s = slice(b * BLOCK, b * BLOCK + m)
        q[s], hi[s], lo[s] = qb, hb, lb
    cfg = osmaq.SmaqConfig(num_bits_main=h["num_bits_main"], num_bits_outlier=h["num_bits_outlier"],
                           main_std_dev_threshold=float(F32(h["thr"])))
    # the ranges come from the header (the compressor's fp32 constants)
    cfg_r = _RangesCfg(cfg, F32(h["range_main"]), F32(h["range_outlier"]))
    return osmaq.dequant(q, hi, lo, h["mean"], h["std_dev"], cfg_r, bool(h["flags"] & 1))


class _RangesCfg:
    """A SmaqConfig view with explicit fp32 ranges (those recorded in the stream header)."""

    def __init__(self, cfg, r_main, r_out):
        self._cfg = cfg
        self.range_normal = r_main
        self.range_outlier = r_out

    def __getattr__(self, k):
        return getattr(self._cfg, k)
