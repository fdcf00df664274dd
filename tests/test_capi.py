"""The C-ABI library (no GPU): it loads, exports every function include/smq.h declares, struct
layouts agree, and the host-only functions behave (RNG == oracle, parameter helpers, sample
drawing, multi-tensor plan layout, argument validation without touching the device)."""

import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "smq.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(smq_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from smart_compress_amd import _native as N

    lib = N.lib()
    declared = _declared_functions()
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(N.SIGNATURES), set(declared) ^ set(N.SIGNATURES)
    assert lib.smq_abi_version() == N.SMQ_ABI_VERSION


def test_struct_layouts_match_header():
    """Compile a tiny C program against include/smq.h and compare sizeof/offsetof with ctypes."""
    import subprocess
    import tempfile

    from smart_compress_amd import _native as N

    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "smq.h"
int main(void) {
  printf("%zu %zu\n", sizeof(SmqSizeRecord), offsetof(SmqSizeRecord, n_outlier));
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(SmqSmaqParams),
         sizeof(SmqSmaqStats), sizeof(SmqTensorDesc), sizeof(SmqS2fp8Stats),
         offsetof(SmqSmaqParams, seed), offsetof(SmqSmaqParams, bn_gamma),
         offsetof(SmqSmaqParams, sample_idx), offsetof(SmqSmaqStats, inv_std_clamped),
         offsetof(SmqSmaqStats, quot_check), sizeof(SmqPackedHeader),
         offsetof(SmqPackedHeader, inv_range_main), offsetof(SmqPackedHeader, error),
         offsetof(SmqS2fp8Stats, rng_offset));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "l")
        subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe])
        got = list(map(int, subprocess.check_output([exe]).split()))
    assert got[:2] == [ctypes.sizeof(N.SmqSizeRecord), N.SmqSizeRecord.n_outlier.offset] == [128, 96]
    got = got[2:]
    want = [ctypes.sizeof(N.SmqSmaqParams), ctypes.sizeof(N.SmqSmaqStats),
            ctypes.sizeof(N.SmqTensorDesc), ctypes.sizeof(N.SmqS2fp8Stats),
            N.SmqSmaqParams.seed.offset, N.SmqSmaqParams.bn_gamma.offset,
            N.SmqSmaqParams.sample_idx.offset, N.SmqSmaqStats.inv_std_clamped.offset,
            N.SmqSmaqStats.quot_check.offset, ctypes.sizeof(N.SmqPackedHeader),
            N.SmqPackedHeader.inv_range_main.offset, N.SmqPackedHeader.error.offset,
            N.SmqS2fp8Stats.rng_offset.offset]
    assert got == want
    from oracle import smaq_packed as P  # the oracle's header struct matches the C layout

    assert P.HEADER_BYTES == got[9] and P._HDR.size == got[9]


def test_host_rng_equals_oracle():
    from oracle import rng
    from smart_compress_amd import _native as N

    lib = N.lib()
    for seed in (0, 1, 2**40 + 7, 2**64 - 1):
        for off in (0, 5, 2**32 - 2, 2**33 + 1):
            got = [lib.smq_rng_u32(seed, off + i) for i in range(6)]
            assert got == list(rng.rng_u32(seed, off, 6))


def test_max_values():
    from smart_compress_amd import _native as N

    lib = N.lib()
    assert lib.smq_float_quant_max_value(5, 2) == 57344.0
    assert lib.smq_float_quant_max_value(5, 10) == 65504.0
    assert lib.smq_float_quant_max_value(4, 3) == 240.0
    assert np.float32(lib.smq_float_quant_max_value(8, 7)) == np.float32(3.3895314e38)


def test_draw_samples():
    from smart_compress_amd import _native as N

    lib = N.lib()
    q = N.SmqSmaqParams()
    lib.smq_smaq_params_init(q)
    assert q.range_std_coef < 0  # "library computes C"; 0.0 is a real coefficient (fp16, n>65504)
    seen = set()
    for off in range(50):
        p = N.SmqSmaqParams()
        lib.smq_smaq_params_init(p)
        p.seed, p.offset = 9, off * 1000
        assert lib.smq_smaq_draw_samples(p, 1000, 16) == 0
        idx = list(p.sample_idx[: p.num_samples])
        assert p.num_samples == 16 and len(set(idx)) == 16 and all(0 <= i < 1000 for i in idx)
        seen.update(idx)
    assert len(seen) > 400  # covers the range
    p = N.SmqSmaqParams()
    lib.smq_smaq_params_init(p)
    assert lib.smq_smaq_draw_samples(p, 10, 16) == 0 and p.num_samples == 10
    assert sorted(p.sample_idx[:10]) == list(range(10))
    assert lib.smq_smaq_draw_samples(p, 1000, 65) != 0
    assert b"SMQ_MAX_SAMPLES" in lib.smq_last_error()


@pytest.mark.parametrize("n,k", [(1000, 16), (10, 16), (64, 64), (2**40, 64), (17, 17), (5, 1)])
def test_draw_samples_equals_oracle_floyd(n, k):
    """The host mirror of the device draw (smq_smaq_draw_samples) and oracle/rng.py floyd_indices
    give the same indices in the same order, for positions beyond 2^32 too."""
    from oracle import rng
    from smart_compress_amd import _native as N

    lib = N.lib()
    for seed, pos in ((9, 0), (2**63 + 5, 2**33 + 7), (1, 123456789)):
        p = N.SmqSmaqParams()
        lib.smq_smaq_params_init(p)
        p.seed, p.offset = seed, pos
        assert lib.smq_smaq_draw_samples(p, n, k) == 0
        got = list(p.sample_idx[: p.num_samples])
        want = rng.floyd_indices(seed, pos, n, k)
        assert got == want.tolist()
        assert len(set(got)) == min(n, k) and all(0 <= i < n for i in got)


def test_oracle_floyd_large_k_distinct_and_uniform():
    """k up to SMQ_MAX_DEVICE_SAMPLES: distinct, in range, k == n is a permutation, and each
    index is drawn with probability ~k/n."""
    from oracle import rng

    idx = rng.floyd_indices(3, 0, 4096, 4096)
    assert sorted(idx.tolist()) == list(range(4096))
    counts = np.zeros(1000)
    for pos in range(400):
        i = rng.floyd_indices(11, pos * 1000, 1000, 100)
        assert len(set(i.tolist())) == 100
        counts[i] += 1
    assert abs(counts.mean() - 40.0) < 1e-9 and counts.std() < 10  # binomial sd ~6


def test_validation_errors_without_device():
    from smart_compress_amd import _native as N

    lib = N.lib()
    p = N.SmqSmaqParams()
    lib.smq_smaq_params_init(p)
    assert lib.smq_smaq_apply_f32(None, None, 0, p, None, None, None, 0, None) == N.SMQ_STATS_SAMPLED * -1
    assert b"n must be >= 1" in lib.smq_last_error()
    assert lib.smq_smaq_stats_f32(None, 10, p, None, 0, None) == -1
    assert lib.smq_float_quant_f32(None, None, 5, 5, 2, 1, 1, None, 0, 0, None) == -1
    assert lib.smq_float_quant_f32(None, None, 0, 9, 2, 1, 1, None, 0, 0, None) == -1
    assert b"exp_bits" in lib.smq_last_error()
    assert lib.smq_s2fp8_roundtrip_f32(None, None, 0, 1, None, 0, 0, None, None, 0, None) == -1
    fake = ctypes.c_void_p(4096)  # never dereferenced: argument checks come first
    assert lib.smq_s2fp8_roundtrip(fake, N.SMQ_DTYPE_F16, fake, 8, 32, 1, None, 0, 0, None, None,
                                   None, 0, None) == -1  # qtorch's kernels take fp32 only
    assert b"precision 32" in lib.smq_last_error()
    assert lib.smq_s2fp8_roundtrip(fake, N.SMQ_DTYPE_F32, fake, 8, 8, 1, None, 0, 0, None, None,
                                   None, 0, None) == -1
    assert lib.smq_s2fp8_roundtrip(fake, 7, fake, 8, 16, 1, None, 0, 0, None, None, None, 0,
                                   None) == -1
    assert lib.smq_float_quant(fake, 5, fake, 0, 8, 5, 2, 1, 1, None, 0, 0, None, None) == -1
    assert lib.smq_float_quant(fake, 0, fake, 2, 8, 5, 2, 1, 1, None, 0, 0, None, None) == -1
    assert b"dtype_out" in lib.smq_last_error()
    assert lib.smq_smaq_params_set(p, 6, 8, 1.0, 1.0, 32) == -1


def test_multi_plan_layout():
    """Plan = header, descriptors, the apply map (4096-element chunks) and the statistics map: per
    tensor up to 8,388,611 elements, runs of whole partials of the single-tensor partition
    (csrc/smaq_small.h: V groups of 4 per lane of 1024, G partials), runs of 4 / V partials
    (V <= 4, else 1) per 1024-thread statistics workgroup; larger tensors have no record (their statistics are the
    single-tensor launch)."""
    from smart_compress_amd import _native as N

    lib = N.lib()
    C = 4096  # default apply chunk (csrc/smaq_multi.hip)
    sizes = [10, C, C + 1, 3 * C + 5, 65537, 300000, 9 << 20]
    count = len(sizes)
    arr = (ctypes.c_int64 * count)(*sizes)
    nbytes = lib.smq_smaq_multi_plan_bytes(arr, count)
    chunks = [-(-n // C) for n in sizes]
    nl = chunks[4]
    # partials G = ceil((n // 4) / 1024) (V = 1 below 2^20 groups); 4 / V = 4 per workgroup
    parts = [1, 1, 1, 4, 16, 74]
    wgs = [-(-g // 4) for g in parts]
    dbytes = ((40 * count + 31) // 32) * 32
    tab = (4 * count + 63) // 64 * 64  # per tensor: its first statistics record to finalize
    assert nbytes == 32 + dbytes + 64 * (sum(chunks) + sum(wgs)) + tab
    descs = (N.SmqTensorDesc * count)()
    rel = 0
    for i, n in enumerate(sizes):
        descs[i].x = descs[i].y = 0x1000 * (i + 1)
        descs[i].n = n
        descs[i].all_positive = i % 2
        descs[i].rng_offset = rel
        rel += n
    host = (ctypes.c_uint8 * nbytes)()
    assert lib.smq_smaq_multi_plan_build(descs, count, host, nbytes) == 0
    raw = np.frombuffer(bytes(host), dtype=np.uint8)
    assert list(raw[:8].view(np.int32)) == [count, sum(chunks)]
    assert int(raw[8:16].view(np.int64)[0]) == C
    assert list(raw[16:24].view(np.int32)) == [sum(wgs), sum(parts)]
    assert int(raw[24:32].view(np.int64)[0]) == 0
    rec = raw[32 + dbytes:nbytes - tab].reshape(-1, 64)
    assert rec.shape[0] == sum(chunks) + sum(wgs)
    fin = raw[nbytes - tab:nbytes - tab + 4 * count].view(np.int32)
    firsts = [sum(wgs[:t]) for t in range(len(wgs))]
    assert list(fin) == [firsts[t] if parts[t] > 1 else -1 for t in range(len(parts))] + [-1]
    q = rec[:, :48].copy().view(np.int64)  # x, y, n, begin, end, rng_offset
    i32 = rec[:, 48:].copy().view(np.int32)  # tensor, first_chunk, n_chunks, all_positive
    a = slice(0, 8 + nl)
    assert list(i32[a, 0]) == [0, 1, 2, 2, 3, 3, 3, 3] + [4] * nl
    assert list(i32[a, 1]) == [0, 1, 2, 2, 4, 4, 4, 4] + [8] * nl
    assert list(i32[a, 2]) == [1, 1, 2, 2, 4, 4, 4, 4] + [nl] * nl
    assert list(i32[a, 3]) == [0, 1, 0, 0, 1, 1, 1, 1] + [0] * nl
    assert list(q[a, 3])[:8] == [0, 0, 0, C, 0, C, 2 * C, 3 * C]
    assert list(q[a, 4])[:8] == [10, C, C, C + 1, C, 2 * C, 3 * C, 3 * C + 5]
    assert list(q[a, 5])[:5] == [0, 10, 10 + C, 10 + C, 10 + 2 * C + 1]
    b = slice(sum(chunks), None)  # the statistics map: partial runs [begin, end)
    tens = [t for t, w in enumerate(wgs) for _ in range(w)]
    first = [sum(parts[:t]) for t in tens]  # first partial of the tensor
    assert list(i32[b, 0]) == tens
    assert list(i32[b, 1]) == first
    assert list(i32[b, 2]) == [wgs[t] for t in tens]
    assert list(q[b, 3]) == [4 * c for w in wgs for c in range(w)]
    assert list(q[b, 4]) == [min(4 * c + 4, g) for g, w in zip(parts, wgs) for c in range(w)]
    assert lib.smq_smaq_multi_workspace_bytes(arr, count) >= 64 * count + 32 * sum(parts)
    descs[1].n = 0
    assert lib.smq_smaq_multi_plan_build(descs, count, host, nbytes) == -1


def test_integration_doc_binding_matches_the_library_struct():
    """INTEGRATION.md's ctypes mirror of SmqSmaqParams (the binding a maintainer copies into
    smart.py) has the library's field names, offsets and size: a short mirror would let the library
    read offset_counter from past the end of the caller's struct."""
    import ctypes as C

    from smart_compress_amd import _native as N

    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = re.search(r"class SmqSmaqParams\(ctypes.Structure\):.*?\)\][^\n]*\n", doc, flags=re.S).group(0)
    ns = {"ctypes": C}
    exec(block, ns)
    mirror = ns["SmqSmaqParams"]
    assert C.sizeof(mirror) == C.sizeof(N.SmqSmaqParams)
    lib_fields = [(f[0], getattr(N.SmqSmaqParams, f[0]).offset) for f in N.SmqSmaqParams._fields_]
    doc_fields = [(f[0], getattr(mirror, f[0]).offset) for f in mirror._fields_]
    assert doc_fields == lib_fields
    # the ratio-logging record mirror (round 6) likewise
    block = re.search(r"class SmqSizeRecord\(ctypes.Structure\):.*?\)\][^\n]*\n", doc, flags=re.S).group(0)
    exec(block, ns)
    rec = ns["SmqSizeRecord"]
    assert C.sizeof(rec) == C.sizeof(N.SmqSizeRecord) == 128
    assert [(f[0], getattr(rec, f[0]).offset) for f in rec._fields_] == \
        [(f[0], getattr(N.SmqSizeRecord, f[0]).offset) for f in N.SmqSizeRecord._fields_]


def test_shipped_library_reads_no_environment():
    """The measurement knobs (SMQ_STATS_GRID, SMQ_DEFER_MAX_N, SMQ_MULTI_RUNS, ...) change
    launch shapes and reduction orders; the shipped library is built without them (smq_common.h
    knob_env): it imports no getenv and holds none of their names."""
    import subprocess

    from smart_compress_amd import _native as N

    syms = subprocess.run(["nm", "-D", "--undefined-only", N.LIB_PATH], capture_output=True,
                          text=True, check=True).stdout
    assert "getenv" not in syms
    blob = open(N.LIB_PATH, "rb").read()
    for knob in (b"SMQ_STATS_GRID", b"SMQ_STATS_PER_WG", b"SMQ_DEFER_MAX_N",
                 b"SMQ_MULTI_RUNS", b"SMQ_MULTI_CHUNK", b"SMQ_FUSED", b"SMQ_CPU_THREADS"):
        assert knob not in blob, knob


def test_fastcall_binding_loads_next_to_the_library():
    """The CPython fast-call binding of smq_smaq_roundtrip (csrc/pyfast.cpp) is built next to
    libsmq.so and calls that same library: a bad argument count raises, and a call with a NULL
    params block returns the library's status (no launch: the library validates first)."""
    from smart_compress_amd import _native as N

    f = N.fast()
    assert f is not None and callable(f.smaq_roundtrip)
    with pytest.raises(TypeError):
        f.smaq_roundtrip(1, 2, 3)
    rc = f.smaq_roundtrip(0, 0, 0, 16, 0, 0, 0, 0)
    assert rc != 0 and N.lib().smq_last_error()


def test_smaq_draws_match_oracle():
    """smq_smaq_u24 (the SmaQ rounding draw: one hash per four counters) equals oracle/rng.py
    smaq_u24 for every alignment of the stream position, across the 2^32 counter boundary and for
    64-bit counters."""
    from oracle import rng
    from smart_compress_amd import _native as N

    lib = N.lib()
    for seed in (0, 1, 2**63 + 5):
        for off in (0, 1, 2, 3, 2**32 - 6, 2**34 + 1, 2**64 - 16):
            got = [lib.smq_smaq_u24(seed, off + i) for i in range(8)]
            assert got == [int(v) for v in rng.smaq_u24(seed, off, 8)]
            assert all(g < 2**24 for g in got)
