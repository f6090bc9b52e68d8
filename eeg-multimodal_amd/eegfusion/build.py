"""Build the HIP C-ABI library ``libeegfusion.so`` in-tree for gfx950.

Each ``csrc/*.hip`` file is compiled separately (in parallel) with ``hipcc --offload-arch=gfx950``
and linked into ``eegfusion/libeegfusion.so``.  Rebuilds are incremental on source/header mtimes.
Run ``python -m eegfusion.build`` (with ``eeg-multimodal_amd`` on ``sys.path``) or call
``build()``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent                    # eeg-multimodal_amd/
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"
OBJ_DIR = ROOT / "build"
LIB_PATH = PKG_DIR / "libeegfusion.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast",
          "-Wno-unused-result", "-Wno-inline-asm", f"-I{INCLUDE}", f"-I{CSRC}"]
# -Wno-inline-asm: the LDS-DMA asm (common.h glds16_asm) lists m0 as clobbered on purpose


def _headers() -> list[Path]:
    return sorted(CSRC.glob("*.h")) + sorted(CSRC.glob("*.inc")) + sorted(INCLUDE.glob("*.h"))


def _needs(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, hdrs: list[Path], verbose: bool) -> Path:
    obj = OBJ_DIR / (src.stem + ".o")
    if _needs(obj, [src, *hdrs]):
        cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    OBJ_DIR.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    hdrs = _headers()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdrs, verbose), srcs))
    if _needs(LIB_PATH, objs):
        # link to a temporary name; only a library that passed the lint is renamed into place, so a
        # lint that fails or cannot run (missing llvm tools) never leaves an unchecked, up-to-date-looking
        # LIB_PATH behind
        tmp = LIB_PATH.with_name(LIB_PATH.name + ".tmp")
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            tmp.unlink(missing_ok=True)
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        try:
            _lint(tmp)
        except BaseException:
            tmp.unlink(missing_ok=True)
            raise
        tmp.replace(LIB_PATH)
    return LIB_PATH


def _lint(lib: Path) -> None:
    """The post-link ISA lint (tools/isa_lint.py) as a failing build step: the hand-written LDS-DMA asm
    relies on wait states hipcc never inserts inside asm (a VALU-written SGPR base read within 5 states,
    an M0 write within 1, a sign-extended address word), so a library with any such site is renamed
    aside and the build fails instead of shipping it."""
    tool = ROOT.parent / "tools" / "isa_lint.py"
    if not tool.exists():              # a package copied without the repository's tools/
        return
    import importlib.util
    spec = importlib.util.spec_from_file_location("eegf_isa_lint", tool)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod           # the tool's dataclasses resolve their module by name
    spec.loader.exec_module(mod)
    findings, _ = mod.lint(lib)
    if findings:
        bad = LIB_PATH.with_name(LIB_PATH.name + ".hazards")
        lib.replace(bad)
        head = "\n".join(f"  {f.kind}: {f.func} @0x{f.addr:x}: '{f.inst}' {f.states} state(s) after '{f.writer}'"
                          for f in findings[:10])
        raise RuntimeError(f"ISA lint: {len(findings)} hazard site(s) in {lib.name} (moved to {bad.name}):\n{head}")


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
