"""Process-global singletons (reference: smart_compress/util/globals.py:5-7).

The reference imports pytorch_lightning only for the profiler's type annotation; here any object
with a ``profile(name)`` context manager works, and ``None`` (no profiler) is tolerated — the
reference would crash on ``Globals.profiler.profile("smaq")`` (smart.py:119) without a Trainer.
"""

import contextlib


class Globals:
    compression = None
    profiler = None


_NO_PROFILER = contextlib.nullcontext()  # reusable: entered once per codec call when no profiler


def profile(name: str):
    prof = Globals.profiler
    if prof is None:
        return _NO_PROFILER
    return prof.profile(name)
