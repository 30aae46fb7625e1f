"""Build a variant of the HIP module with extra compiler flags for same-box A/B runs:

    python scripts/build_variant.py NAME [-DFLAG ...]

writes build/ab/NAME/_tts_hip<EXT> (the kernels recompiled with the flags, the bindings
object shared); scripts/ab_so.sh swaps variants into the package on the GPU box. With no
flags, NAME is a copy of the current module (the A side)."""
import shutil
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from dist_gpu_accelerated_tree_search_amd.ops import build as B  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out_dir = B.BUILD / "ab" / name
out_dir.mkdir(parents=True, exist_ok=True)
out = out_dir / f"_tts_hip{B.EXT}"
newest = B._sources_mtime()
B.build_hip(newest, 8)  # the A side and the shared bindings object are current
if not flags:
    shutil.copy2(B.hip_module_path(), out)
else:
    B.OBJ = out_dir / "obj"
    B.HIPFLAGS = [*B.HIPFLAGS, *flags]
    B._HIP_OBJS = None
    objs = B._hip_objects(newest, 8)
    B._run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", str(B.BUILD / "obj" / "py_hip.o"),
            *map(str, objs), *B.HIP_MODULE_LIBS, "-o", str(out)])
print(out)
