"""Native extension loaders.

``cpu()`` returns the host core module (g++ build, always available after
``ops.build``). ``hip()`` returns the gfx950 device module and raises loudly when it
is missing or when no GPU is visible — there is no silent PyTorch/CPU fallback for
GPU paths.
"""
from __future__ import annotations

import importlib
import os

_cpu_mod = None
_hip_mod = None


class NativeExtensionMissing(ImportError):
    pass


def _import(name: str):
    try:
        return importlib.import_module(f"dist_gpu_accelerated_tree_search_amd.{name}")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise NativeExtensionMissing(
            f"native extension {name} is not built; run `python -m dist_gpu_accelerated_tree_search_amd.ops.build` "
            f"(or __graft_entry__.build()). Import error: {e}"
        ) from e


def cpu():
    global _cpu_mod
    if _cpu_mod is None:
        if os.environ.get("TTS_AUTOBUILD", "1") == "1":
            _maybe_build("cpu")
        _cpu_mod = _import("_tts_cpu")
    return _cpu_mod


def hip():
    """The HIP module. Raises if it is not built or no device is visible.

    torch (when installed) is imported first: its bundled libamdhip64 carries the
    same SONAME as /opt/rocm's, so loading it first makes the extension bind to the
    one HIP runtime torch uses (device pointers and streams are then shared);
    loading ours first would put two HIP runtimes in one process.
    """
    global _hip_mod
    if _hip_mod is None:
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - torch is part of the stack
            pass
        if os.environ.get("TTS_AUTOBUILD", "1") == "1":
            _maybe_build("hip")
        _hip_mod = _import("_tts_hip")
    return _hip_mod


def gpu_count() -> int:
    """Number of visible GPUs without initialising HIP in this process (torch's
    device_count does not initialise the runtime on this image)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover
        return 0


def require_gpu(device: int = 0):
    m = hip()
    n = m.device_count()
    if n <= device:
        raise RuntimeError(f"GPU {device} requested but only {n} HIP device(s) are visible")
    return m


def _maybe_build(which: str) -> None:
    from . import build as _b

    target = _b.cpu_module_path() if which == "cpu" else _b.hip_module_path()
    if target.exists():  # explicit `ops.build` refreshes stale modules; imports never do
        return
    try:
        _b.build_all(only=which)
    except Exception as e:  # keep an existing (older) module usable; raise only if none
        if not target.exists():
            raise NativeExtensionMissing(f"building {which} extension failed: {e}") from e
