"""TEST INFRASTRUCTURE ONLY — the counter-based RNG of libsmq, restated in numpy (bit-exact with
smq_common.h: mix32, rng_key, rng_u32, mix32x3 / quad_word / draw_mul / smaq_u24). Element i of a call with (seed,
offset) uses counter offset + i: the float quantiser draws rng_u32(counter) per element, SmaQ's
stochastic rounding smaq_u24(counter) — one hash per four consecutive counters."""

import numpy as np

_M32 = 0xFFFFFFFF


def mix32(x):
    x = np.asarray(x, dtype=np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def mix32x3(x):
    """triple32 (smq_common.h mix32x3): the quad hash of SmaQ's draws."""
    x = np.asarray(x, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(17)
        x *= np.uint32(0xED5AD4BB)
        x ^= x >> np.uint32(11)
        x *= np.uint32(0xAC4C1B51)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x31848BAB)
        x ^= x >> np.uint32(14)
    return x


def _mix32_int(v: int) -> int:
    return int(mix32(np.array([v & _M32], dtype=np.uint32))[0])


def rng_key(seed: int) -> int:
    seed &= (1 << 64) - 1
    return _mix32_int((seed & _M32) ^ _mix32_int(((seed >> 32) ^ 0x9E3779B9) & _M32))


def rng_u32(seed: int, offset: int, n: int, start: int = 0) -> np.ndarray:
    """Random words for elements start..start+n-1 of a call keyed by (seed, offset)."""
    key = np.uint32(rng_key(seed))
    ctr = (np.uint64(offset) + np.arange(start, start + n, dtype=np.uint64))
    lo = (ctr & np.uint64(_M32)).astype(np.uint32)
    hi = (ctr >> np.uint64(32)).astype(np.uint32)
    rot = (hi << np.uint32(16)) | (hi >> np.uint32(16))
    return mix32(lo ^ rot ^ key)


def u32_to_unit(h: np.ndarray) -> np.ndarray:
    return (h >> np.uint32(8)).astype(np.float32) * np.float32(2.0**-24)


DRAW_MUL = np.array([1, 0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D], dtype=np.uint32)


def smaq_u24(seed: int, offset: int, n: int, start: int = 0) -> np.ndarray:
    """SmaQ's draws (smq_common.h smaq_u24) for elements start..start+n-1 of a call keyed by
    (seed, offset): quad word h = mix32x3(lo ^ rotl16(hi) ^ key) of q = counter >> 2, lane
    counter & 3 takes the top 24 bits of h * DRAW_MUL[lane] (uint32 wrap-around)."""
    key = np.uint32(rng_key(seed))
    ctr = (np.uint64(offset) + np.arange(start, start + n, dtype=np.uint64))
    q = ctr >> np.uint64(2)
    lo = (q & np.uint64(_M32)).astype(np.uint32)
    hi = (q >> np.uint64(32)).astype(np.uint32)
    rot = (hi << np.uint32(16)) | (hi >> np.uint32(16))
    h = mix32x3(lo ^ rot ^ key)
    with np.errstate(over="ignore"):
        return (h * DRAW_MUL[(ctr & np.uint64(3)).astype(np.intp)]) >> np.uint32(8)


def uniforms(seed: int, offset: int, n: int, start: int = 0) -> np.ndarray:
    """SmaQ's stochastic-rounding uniforms (smaq_u24 * 2^-24), fp32."""
    return smaq_u24(seed, offset, n, start).astype(np.float32) * np.float32(2.0**-24)


DRAW_SALT = 0xD1B54A32D192ED03


def floyd_indices(seed: int, position: int, n: int, k: int) -> np.ndarray:
    """The k = min(n, num_samples) distinct sample indices libsmq draws for SMQ_STATS_SAMPLED_DEVICE
    at stream position ``position`` (smaq.hip smaq_draw_stats_kernel / smq_smaq_draw_samples), in
    draw order — the stand-in for the reference's ``torch.randperm(n)[:k]`` (smart.py:88).
    Floyd's algorithm: step i (j = n - k + i) takes t = h_i mod (j + 1), or j if t was taken, with
    h_i = (u32(2P + 2i) << 32) | u32(2P + 2i + 1) under the key rng_key(seed ^ DRAW_SALT)."""
    k = min(int(n), int(k))
    salted = (int(seed) ^ DRAW_SALT) & ((1 << 64) - 1)
    key = rng_key(salted)
    ctr = (2 * int(position) + np.arange(2 * k, dtype=np.uint64)) & np.uint64((1 << 64) - 1)
    lo = (ctr & np.uint64(_M32)).astype(np.uint32)
    hi = (ctr >> np.uint64(32)).astype(np.uint32)
    rot = (hi << np.uint32(16)) | (hi >> np.uint32(16))
    w = mix32(lo ^ rot ^ np.uint32(key)).astype(np.uint64)
    h = (w[0::2] << np.uint64(32)) | w[1::2]
    out, taken = [], set()
    for i in range(k):
        j = n - k + i
        t = int(h[i] % np.uint64(j + 1))
        if t in taken:
            t = j
        taken.add(t)
        out.append(t)
    return np.array(out, dtype=np.int64)
