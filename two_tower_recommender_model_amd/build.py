"""Build recipe of libtt_mi355x.so (gfx950 only), compiled in-tree with hipcc.

    python -m two_tower_recommender_model_amd.build          # incremental
    python -m two_tower_recommender_model_amd.build --force

Each translation unit is compiled to an object in ``build/`` (parallel), then linked into
``two_tower_recommender_model_amd/lib/libtt_mi355x.so``. The library travels to the GPU box with the
repository snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
BUILD = ROOT / "build" / "tt_mi355x"
LIB = PKG / "lib" / "libtt_mi355x.so"
# experiment build (stamps / debug bits compiled in; loaded only with TT_EXPERIMENT_LIB=1)
BUILD_EXP = ROOT / "build" / "tt_mi355x_exp"
LIB_EXP = PKG / "lib_exp" / "libtt_mi355x.so"
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["api.cpp", "kjt.hip", "embedding.hip", "gemm.hip", "loss_adam.hip", "tower.hip", "dedup.hip", "shard.hip", "shard_kjt.hip", "peer.hip"]
HEADERS = [CSRC / "tt_common.h", CSRC / "dedup.h", CSRC / "shard.h", INCLUDE / "tt_mi355x.h"]

CFLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-munsafe-fp-atomics",
    f"-I{INCLUDE}",
    f"-I{CSRC}",
    "-Wall",
    "-Wno-unused-function",
]
# experiment-only extra flags (e.g. -DDD_HOT_STAMPS=1); applied to the --experiments build only
EXTRA_EXP = os.environ.get("TT_EXTRA_CFLAGS", "").split()


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path, extra=()) -> None:
    cmd = [HIPCC, *CFLAGS, *extra, "-x", "hip", "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, verbose: bool = False, experiments: bool = False) -> Path:
    bdir, lib_path = (BUILD_EXP, LIB_EXP) if experiments else (BUILD, LIB)
    if EXTRA_EXP and not experiments:
        raise RuntimeError("TT_EXTRA_CFLAGS is for the experiment build only: add --experiments "
                           "(the release lib/ is always built from the tree as committed)")
    extra = ["-DTT_EXPERIMENTS=1", *EXTRA_EXP] if experiments else []
    if experiments and EXTRA_EXP:
        force = True  # objects do not record their flags: rebuild when extra flags are given
    bdir.mkdir(parents=True, exist_ok=True)
    lib_path.parent.mkdir(parents=True, exist_ok=True)
    objs = []
    jobs = []
    for s in SOURCES:
        src = CSRC / s
        obj = bdir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *HEADERS]):
            jobs.append((src, obj))
    if jobs:
        workers = min(len(jobs), max(1, min(8, os.cpu_count() or 1)))
        with cf.ThreadPoolExecutor(workers) as ex:
            futs = [ex.submit(_compile, s, o, extra) for s, o in jobs]
            for f in futs:
                f.result()
        if verbose:
            print("compiled:", ", ".join(s.name for s, _ in jobs))
    if force or jobs or _stale(lib_path, objs):
        tmp = lib_path.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, lib_path)
        if verbose:
            print("linked", lib_path)
    return lib_path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--experiments", action="store_true", help="stamps / debug bits compiled in (lib_exp/)")
    args = ap.parse_args()
    try:
        build(force=args.force, verbose=True, experiments=args.experiments)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
