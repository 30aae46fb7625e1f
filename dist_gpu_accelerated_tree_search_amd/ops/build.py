"""In-tree build of the native pieces (no setuptools, no JIT cache).

Targets (all written inside the repository so they travel with it):
  dist_gpu_accelerated_tree_search_amd/_tts_cpu*.so   g++   host core + CPU drivers
  dist_gpu_accelerated_tree_search_amd/_tts_hip*.so   hipcc gfx950 kernels + device engines
  build/bin/{pfsp_c,pfsp_omp_c,nqueens_c}             g++   native CLIs (ref *_c.c)
  build/bin/{pfsp_gpu,nqueens_gpu}                    hipcc native single-process GPU CLIs

Parity: replaces ref pfsp/makefile + CMakeLists.txt (nvcc / hipify-perl + hipcc for
gfx906/gfx90a/gfx1102) with one gfx950-only HIP build.

Usage: python -m dist_gpu_accelerated_tree_search_amd.ops.build [--only cpu|hip|cli] [-j N]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build"
OBJ = BUILD / "obj"
BIN = BUILD / "bin"
ARCH = os.environ.get("TTS_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX_HOST", "g++")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-maybe-uninitialized", "-Wno-unused-function"]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIP_LIBS = [f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lrocprofiler-sdk-roctx"]
# the Python module also links librccl.so.1 (csrc/hip/rccl_transport.hpp): a process
# that imported torch first already holds torch's copy (same SONAME), so one RCCL per process
HIP_MODULE_LIBS = [*HIP_LIBS, "-lrccl"]
HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _sources_mtime() -> float:
    return max(p.stat().st_mtime for p in CSRC.rglob("*") if p.is_file())


def _stale(out: Path, newest: float) -> bool:
    return not out.exists() or out.stat().st_mtime < newest


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd[:3])} ... {cmd[-1]}")


def cpu_module_path() -> Path:
    return PKG / f"_tts_cpu{EXT}"


def hip_module_path() -> Path:
    return PKG / f"_tts_hip{EXT}"


def build_cpu(newest: float) -> Path:
    out = cpu_module_path()
    if _stale(out, newest):
        _run([CXX, *CXXFLAGS, "-shared", *_py_includes(), str(CSRC / "bindings" / "py_cpu.cpp"), "-o", str(out)])
    return out


def build_cli(newest: float, jobs: int, with_hip: bool = True) -> list[Path]:
    BIN.mkdir(parents=True, exist_ok=True)
    tasks = []
    for name in ("pfsp_c", "pfsp_omp_c", "nqueens_c"):
        out = BIN / name
        if _stale(out, newest):
            tasks.append([CXX, *CXXFLAGS, str(CSRC / "apps" / f"{name}.cpp"), "-o", str(out)])
    if with_hip:
        for name in ("pfsp_gpu", "nqueens_gpu"):
            src = CSRC / "apps" / f"{name}.hip"
            out = BIN / name
            if src.exists() and _stale(out, newest):
                objs = [str(o) for o in _hip_objects(newest, jobs)]
                app_o = OBJ / f"app_{name}.o"
                tasks.append([[HIPCC, *HIPFLAGS, "-pthread", "-c", str(src), "-o", str(app_o)],
                              [HIPCC, f"--offload-arch={ARCH}", "-pthread", str(app_o), *objs, *HIP_LIBS, "-o",
                               str(out)]])
    def run_task(t):
        for c in (t if isinstance(t[0], list) else [t]):
            _run(c)

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(run_task, tasks))
    return [BIN / n for n in ("pfsp_c", "pfsp_omp_c", "nqueens_c", "pfsp_gpu", "nqueens_gpu")]


_HIP_OBJS: list[Path] | None = None


def _hip_objects(newest: float, jobs: int) -> list[Path]:
    """Kernel/engine translation units (shared by the Python module and the CLIs)."""
    global _HIP_OBJS
    if _HIP_OBJS is not None:
        return _HIP_OBJS
    OBJ.mkdir(parents=True, exist_ok=True)
    srcs = sorted((CSRC / "hip").glob("*.hip"))
    tasks, objs = [], []
    for s in srcs:
        o = OBJ / (s.stem + ".o")
        objs.append(o)
        if _stale(o, newest):
            tasks.append([HIPCC, *HIPFLAGS, "-c", str(s), "-o", str(o)])
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, tasks))
    _HIP_OBJS = objs
    return objs


def build_hip(newest: float, jobs: int) -> Path:
    out = hip_module_path()
    objs = _hip_objects(newest, jobs)
    bind_o = OBJ / "py_hip.o"
    if _stale(bind_o, newest):
        _run([HIPCC, *HIPFLAGS, "-x", "hip", *_py_includes(), "-c", str(CSRC / "bindings" / "py_hip.cpp"), "-o",
              str(bind_o)])
    if _stale(out, newest):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", str(bind_o), *map(str, objs), *HIP_MODULE_LIBS, "-o",
              str(out)])
    return out


SANITIZERS = {"tsan": ["-fsanitize=thread"], "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]}


def build_sanitized_selftests(kinds=("tsan", "asan"), jobs: int = 2) -> dict[str, Path]:
    """Host runtime self-test (csrc/tests/runtime_selftest.cpp) under TSan and
    ASan+UBSan. Host code only: GPU sanitizers are not used."""
    BIN.mkdir(parents=True, exist_ok=True)
    src = CSRC / "tests" / "runtime_selftest.cpp"
    newest = _sources_mtime()
    tasks, outs = [], {}
    for k in kinds:
        out = BIN / f"runtime_selftest_{k}"
        outs[k] = out
        if _stale(out, newest):
            tasks.append([CXX, "-O1", "-g", "-std=c++17", "-pthread", *SANITIZERS[k], f"-I{CSRC}", str(src), "-o",
                          str(out)])
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, tasks))
    return outs


def build_all(only: str | None = None, jobs: int | None = None) -> dict[str, Path]:
    jobs = jobs or min(16, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
    newest = _sources_mtime()
    res: dict[str, Path] = {}
    if only in (None, "cpu"):
        res["cpu"] = build_cpu(newest)
    if only in (None, "hip"):
        res["hip"] = build_hip(newest, jobs)
    if only in (None, "cli"):
        for p in build_cli(newest, jobs):
            res[p.name] = p
    return res


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--only", choices=["cpu", "hip", "cli"])
    ap.add_argument("-j", "--jobs", type=int)
    a = ap.parse_args(argv)
    for k, v in build_all(a.only, a.jobs).items():
        print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
