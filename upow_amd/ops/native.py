"""Loader for the in-tree native extension (``upow_amd/_native*.so``).

The extension holds the host C++ crypto and the gfx950 HIP kernels. There is no silent Python
fallback on a GPU box: :func:`lib` raises if the extension is missing, and :func:`gpu_available`
reports whether a HIP device is usable (so CPU-only containers take the host C++ path explicitly).
Set ``UPOW_AUTOBUILD=1`` to build on first import.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_lib = None
_gpu = None


def _preload_torch_hip():
    """Make the process use ONE HIP runtime.

    The PyTorch-ROCm wheel ships its own ``libamdhip64.so`` (SONAME ``libamdhip64.so.7``) and its
    libraries NEED it by file name; our extension NEEDS ``libamdhip64.so.7``. Loading torch first
    makes the dynamic loader resolve our dependency to torch's already-loaded runtime (SONAME match),
    so torch tensors/streams/RCCL and our kernels share one HIP context. Loading ours first would map
    /opt/rocm's runtime and torch would then map a second copy.
    """
    if os.environ.get('UPOW_NO_TORCH', '0') == '1':
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _preload_torch_hip()
            so = os.environ.get('UPOW_NATIVE_SO')  # an instrumented build (tools/sanitize_host.sh)
            if so:
                import importlib.util as ilu
                import sys
                spec = ilu.spec_from_file_location('upow_amd._native', so)
                _lib = ilu.module_from_spec(spec)
                spec.loader.exec_module(_lib)
                sys.modules['upow_amd._native'] = _lib
                return _lib
            try:
                _lib = importlib.import_module('upow_amd._native')
            except ImportError as e:
                if os.environ.get('UPOW_AUTOBUILD', '0') == '1':
                    from .. import _build
                    _build.build(verbose=False)
                    _lib = importlib.import_module('upow_amd._native')
                else:
                    raise ImportError('upow_amd._native is not built: run `python -m upow_amd._build` '
                                      '(hipcc --offload-arch=gfx950)') from e
    return _lib


def gpu_available() -> bool:
    """True when the extension sees at least one HIP device (does not initialise torch)."""
    global _gpu
    if _gpu is None:
        if os.environ.get('UPOW_DISABLE_GPU', '0') == '1':
            _gpu = False
        else:
            try:
                _gpu = lib().gpu_device_count() > 0
            except Exception:
                _gpu = False
    return _gpu


def require_gpu():
    if not gpu_available():
        raise RuntimeError('no HIP device visible to upow_amd._native')
    return lib()
