"""Build the in-tree HIP extension ``llmtrain/ops/_llmtrain_hip.so`` for gfx950.

    python -m llmtrain.ops.build [--jobs N] [--force] [--debug]
    python -m llmtrain.ops.build --variant NAME -D MACRO[=VALUE] ... [--cflag=-fFLAG]   # A/B build

Every ``csrc/*.hip`` kernel file is compiled by ``hipcc --offload-arch=gfx950`` into its own
object (these TUs include only the HIP runtime, so they compile in seconds); ``csrc/bindings.cpp``
— the only TU that includes torch headers — is compiled once; everything is linked into one
shared object that ``torch.ops.load_library`` loads.  Objects are rebuilt only when a source or
header is newer (incremental).  The build needs no GPU: hipcc cross-compiles for gfx950.

No hipify, no CUDA sources, no multi-arch fat binaries: gfx950 (MI355X, CDNA4) only.
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import torch

__all__ = ["build", "CSRC", "OUT", "OUT_DEBUG"]

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "csrc"
OUT = Path(__file__).resolve().with_name("_llmtrain_hip.so")
# `--debug`: -O1 -g with device-side bounds asserts (LLMT_DASSERT in csrc/common.h); loaded instead
# of the release object when LLMTRAIN_DEBUG_KERNELS=1 (see llmtrain/ops/_ext.py)
OUT_DEBUG = Path(__file__).resolve().with_name("_llmtrain_hip_debug.so")
OBJDIR = REPO / "build" / "hip_obj"
# `--variant NAME -D ...`: the same sources with extra preprocessor defines, linked to
# llmtrain/ops/variants/_llmtrain_hip_NAME.so (in-tree, so it travels to the GPU box) and loaded in
# place of the release object through LLMTRAIN_HIP_EXT — same-box A/B of a kernel change
VARIANTS = Path(__file__).resolve().with_name("variants")
ARCH = "gfx950"  # MI355X (CDNA4) only


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return str(Path(rocm) / "bin" / "hipcc")


def _torch_dirs() -> tuple[Path, Path]:
    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "lib"


def _common_flags(debug: bool) -> list[str]:
    flags = [
        f"--offload-arch={ARCH}",
        "-std=c++17",
        "-fPIC",
        "-O1" if debug else "-O3",
        f"-I{CSRC}",
        "-D__HIP_PLATFORM_AMD__",
        "-Wno-unused-result",
    ]
    if debug:
        flags += ["-g", "-DLLMT_DEBUG=1"]
    return flags


def _torch_flags() -> list[str]:
    inc, _ = _torch_dirs()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return [
        f"-I{inc}",
        f"-I{inc / 'torch' / 'csrc' / 'api' / 'include'}",
        f"-I{sysconfig.get_paths()['include']}",
        "-DUSE_ROCM",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
    ]


def _headers() -> list[Path]:
    return sorted(CSRC.glob("*.h"))


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    mtime = obj.stat().st_mtime
    return any(p.stat().st_mtime > mtime for p in [src, *_headers(), Path(__file__)])


def _compile(src: Path, debug: bool, force: bool, objdir: Path = OBJDIR, defines: tuple[str, ...] = (),
             cflags: tuple[str, ...] = ()) -> Path:
    obj = objdir / (src.name + (".dbg" if debug else "") + ".o")
    if not force and not _stale(obj, src):
        return obj
    cmd = [_hipcc(), *_common_flags(debug), *(f"-D{d}" for d in defines)]
    if src.suffix == ".hip":
        cmd += list(cflags)
    if src.suffix == ".cpp":
        cmd += ["-x", "hip", *_torch_flags()]
    cmd += ["-c", str(src), "-o", str(obj)]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{proc.stdout}\n{proc.stderr}")
    return obj


def build(
    *, jobs: int | None = None, force: bool = False, debug: bool = False, verbose: bool = True,
    variant: str | None = None, defines: tuple[str, ...] = (), cflags: tuple[str, ...] = (),
) -> Path:
    """Compile every kernel for gfx950 and link the extension; returns the .so path."""
    objdir = OBJDIR if variant is None else OBJDIR.parent / f"hip_obj_{variant}"
    objdir.mkdir(parents=True, exist_ok=True)
    sources = sorted(CSRC.glob("*.hip")) + [CSRC / "bindings.cpp"]
    jobs = jobs or min(16, os.cpu_count() or 4, len(sources))
    with ThreadPoolExecutor(max_workers=jobs) as pool:
        objs = list(pool.map(lambda s: _compile(s, debug, force, objdir, defines, cflags), sources))
    newest = max(o.stat().st_mtime for o in objs)
    out = OUT_DEBUG if debug else OUT
    if variant is not None:
        VARIANTS.mkdir(exist_ok=True)
        out = VARIANTS / f"_llmtrain_hip_{variant}.so"
    if force or not out.exists() or out.stat().st_mtime < newest:
        _, lib = _torch_dirs()
        cmd = [
            _hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), f"-L{lib}",
            "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip",
            f"-Wl,-rpath,{lib}", "-o", str(out),
        ]
        proc = subprocess.run(cmd, capture_output=True, text=True)
        if proc.returncode != 0:
            raise RuntimeError(f"link failed:\n{proc.stdout}\n{proc.stderr}")
        if verbose:
            print(f"[llmtrain.ops.build] linked {out} ({out.stat().st_size / 2**20:.1f} MiB, {ARCH})")
    elif verbose:
        print(f"[llmtrain.ops.build] {out} up to date")
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--variant", default=None, help="A/B build name (llmtrain/ops/variants/)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra define for --variant")
    ap.add_argument("--cflag", dest="cflags", action="append", default=[],
                    help="extra hipcc flag for the kernel files of a --variant (e.g. -fno-slp-vectorize)")
    args = ap.parse_args(argv)
    if (args.defines or args.cflags) and args.variant is None:
        ap.error("-D / --cflag need --variant (the release build takes no extra flags)")
    build(jobs=args.jobs, force=args.force or bool(args.defines) or bool(args.cflags), debug=args.debug,
          variant=args.variant, defines=tuple(args.defines), cflags=tuple(args.cflags))
    return 0


if __name__ == "__main__":
    sys.exit(main())
