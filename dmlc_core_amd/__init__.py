"""dmlc-core for MI355X.

A brand-new, MI355X-native distributed-ML data runtime with the capabilities
of dmlc-core: URI streams and filesystems, sharded InputSplits, RecordIO,
LibSVM/LibFM/CSV parsers producing CSR RowBlocks, Parameter/Registry/JSON,
ThreadedIter prefetch, and the dmlc-submit tracker -- plus a GPU ingestion
path (pinned-host ring -> HIP/CDNA4 kernels -> CSR in HBM) and RCCL-based
multi-GPU sharding.

The native runtime lives in ``dmlc_core_amd/lib/libdmlc.so`` (C++17 + HIP for
gfx950) and is exposed through ``dmlc_core_amd._dmlc`` (pybind11).  Build it
with ``make -j8`` (or ``python -c "import __graft_entry__ as g; g.build()"``).

Subpackages load lazily (PEP 562): ``import dmlc_core_amd`` alone touches
neither torch nor the HIP runtime, so a launcher process
(``python -m dmlc_core_amd.parallel.launch.submit``, or ``bench.py --gpus N``
spawning its ranks) never maps ``libamdhip64`` -- only the ranks it starts do.
"""
from __future__ import annotations

import importlib
import importlib.abc
import os
import sys

__version__ = "0.1.0"

_HERE = os.path.dirname(os.path.abspath(__file__))
_SUBMODULES = ("utils", "io", "data", "ops", "parallel", "models")


def _load_native():
    # One HIP runtime per process: PyTorch-ROCm bundles libamdhip64.so.7 (same
    # SONAME as /opt/rocm's).  Loading torch first makes libdmlc.so bind to
    # torch's copy, so device pointers, streams and events are shared; loading
    # /opt/rocm's first would leave torch with "No HIP GPUs are available".
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch is optional for the C++-only path
        pass
    try:
        return importlib.import_module(__name__ + "._dmlc")
    except ImportError as err:  # pragma: no cover - exercised only when unbuilt
        raise ImportError(
            "dmlc_core_amd native extension is not built; run `make -j8` in the repo root "
            f"({err})") from err


class _TorchBeforeNative(importlib.abc.MetaPathFinder):
    """Whichever way the extension is imported (``from dmlc_core_amd._dmlc
    import X`` bypasses the package ``__getattr__``), torch is loaded first."""

    def find_spec(self, fullname, path, target=None):  # noqa: D401
        if fullname == __name__ + "._dmlc" and "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except ImportError:  # pragma: no cover
                pass
        return None  # the regular finders load the module


if not any(isinstance(f, _TorchBeforeNative) for f in sys.meta_path):
    sys.meta_path.insert(0, _TorchBeforeNative())


def __getattr__(name):
    if name == "_dmlc":
        mod = _load_native()
    elif name in _SUBMODULES:
        mod = importlib.import_module(f"{__name__}.{name}")
    else:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    globals()[name] = mod
    return mod


__all__ = list(_SUBMODULES) + ["__version__"]
