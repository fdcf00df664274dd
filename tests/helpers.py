"""Shared test helpers: golden fixture loading, hparams building, C-ABI call wrappers."""

import glob
import json
import os
from argparse import ArgumentParser, Namespace

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def smaq_cases():
    with open(os.path.join(GOLDEN, "smaq_cases.json")) as f:
        return json.load(f)


def float_meta():
    with open(os.path.join(GOLDEN, "float_cases.json")) as f:
        return json.load(f)


def s2p16_meta():
    with open(os.path.join(GOLDEN, "s2fp8_p16_cases.json")) as f:
        return json.load(f)


def load_s2p16(key):
    return dict(np.load(os.path.join(GOLDEN, f"s2p16_{key}.npz")))


def load_smaq(name):
    return dict(np.load(os.path.join(GOLDEN, f"smaq_{name}.npz")))


def load_float(key):
    return dict(np.load(os.path.join(GOLDEN, f"float_{key}.npz")))


def oracle_cfg(meta):
    from oracle import smaq

    return smaq.SmaqConfig(
        num_bits_main=meta["num_bits_main"], num_bits_outlier=meta["num_bits_outlier"],
        main_std_dev_threshold=meta["main_std_dev_threshold"],
        outlier_std_dev_threshold=meta["outlier_std_dev_threshold"],
        stochastic_rounding=meta["stochastic_rounding"],
        use_sample_stats=meta["use_sample_stats"], num_samples=meta["num_samples"],
        use_range_std_dev=meta["use_range_std_dev"], min_size=meta["min_size"],
        precision=meta.get("precision", 32),
    )


def smaq_hparams(meta=None, **over):
    """hparams Namespace for smart_compress_amd's SmartFP from a golden case's metadata."""
    from smart_compress_amd.compress.smart import SmartFP

    hp = SmartFP.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 32
    if meta:
        for k in vars(hp):
            if k in meta:
                setattr(hp, k, meta[k])
    for k, v in over.items():
        setattr(hp, k, v)
    return hp


def same_f32(a, b):
    """Bitwise-equal float32 arrays, with every NaN equal to every NaN."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((a.view(np.uint32) == b.view(np.uint32)) | both_nan))


def n_diff_f32(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    ok = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return int((~ok).sum())


def ulp_diff(a, b):
    a = np.int64(np.array(a, np.float32).view(np.int32))
    b = np.int64(np.array(b, np.float32).view(np.int32))
    return int(abs(a - b))
