"""Loader for the native core (`lib/_nm03*.so` → `lib/libnm03.so`).

torch is imported FIRST when available: torch ships its own libamdhip64.so.7/librccl.so.1 and the
dynamic linker then binds libnm03.so to those same objects (identical SONAMEs), so torch tensors,
torch streams and our kernels share one HIP runtime and one device context.

On a machine with a GPU the extension is mandatory: there is no silent fallback to a Python or
CPU path (`native()` raises). On a CPU-only machine tests can still use the host codecs and the
golden model from the same extension.
"""
import importlib
import os

_NATIVE = None
_ERR = None


def _import_torch_first():
    try:
        import torch  # noqa: F401
        return True
    except Exception:  # pragma: no cover - torch missing
        return False


def native():
    """Return the `_nm03` extension module, building nothing; raises with a clear message."""
    global _NATIVE, _ERR
    if _NATIVE is not None:
        return _NATIVE
    _import_torch_first()
    try:
        _NATIVE = importlib.import_module("nm03_capstone_project_amd.lib._nm03")
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        _ERR = e
        raise ImportError(
            "nm03 native extension not built: run `python build.py` (or __graft_entry__.build()) "
            f"before using the engine ({e})") from e
    return _NATIVE


def available():
    try:
        native()
        return True
    except ImportError:
        return False


def lib_dir():
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
