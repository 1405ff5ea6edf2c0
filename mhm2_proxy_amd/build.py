"""Build the native libraries in-tree (they travel to the GPU box with the repo snapshot).

  mhm2_proxy_amd/libmhmkc.so        hipcc --offload-arch=gfx950: HIP kernels + C ABI (include/mhmkc.h)
  mhm2_proxy_amd/libmhmkc_synth.so  gcc: deterministic synthetic read generator (include/mhmkc_synth.h)
  oracle/liboracle.so (+ _ref/)     make -C oracle: the CPU checker (test infrastructure only)
  tools/bin/kmermap_fill            g++: KmerMap fill timing of the C++ adapter from table files (tests, bench.py)
  tools/bin/libmhmkc_handoff.so     g++: the adapter's streamed hand-off (load_ordered) timed in bench.py's process

Incremental: a target is rebuilt only when one of its sources is newer; libmhmkc.so also when the build id it
carries (the SHA-256 of its sources, mhmkc_build_id) is not the tree's, whatever the file times say.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
ARCH = os.environ.get("MHMKC_OFFLOAD_ARCH", "gfx950")

LIB = PKG / "libmhmkc.so"
SYNTH = PKG / "libmhmkc_synth.so"
ORACLE = ROOT / "oracle" / "liboracle.so"

LIB_SOURCES = [CSRC / "kcount_kernels.hip", CSRC / "kcount_ctg.hip", CSRC / "kcount_owner.hip", CSRC / "fastq.hip",
               CSRC / "mhmkc_host.cpp"]
LIB_DEPS = LIB_SOURCES + [CSRC / "kcount_launch.hpp", CSRC / "kmer_ops.hpp", ROOT / "include" / "mhmkc.h"]
SYNTH_DEPS = [CSRC / "synth.c", ROOT / "include" / "mhmkc_synth.h"]
FILL = ROOT / "tools" / "bin" / "kmermap_fill"
FILL_DEPS = [ROOT / "tools" / "cpp" / "kmermap_fill.cpp", ROOT / "include" / "mhmkc_kcount.hpp", ROOT / "include" / "mhmkc.h"]
HANDOFF = ROOT / "tools" / "bin" / "libmhmkc_handoff.so"
HANDOFF_DEPS = [ROOT / "tools" / "cpp" / "handoff.cpp", ROOT / "include" / "mhmkc_kcount.hpp", ROOT / "include" / "mhmkc.h"]
# test infrastructure: the restated traversal over a given table (the multi-rank multi-k chain, tests/test_c5_scale.py)
DBJG = ROOT / "tools" / "bin" / "libmhmkc_dbjg.so"
DBJG_DEPS = [ROOT / "tools" / "cpp" / "dbjg_lib.cpp", ROOT / "include" / "mhmkc_dbjg.hpp",
             ROOT / "include" / "mhmkc_kcount.hpp", ROOT / "include" / "mhmkc.h"]


def source_build_id() -> str:
    """First 16 hex digits of the SHA-256 over libmhmkc.so's sources (relative path and content of each LIB_DEPS
    file, in order): compiled into the library as mhmkc_build_id()."""
    h = hashlib.sha256()
    for d in LIB_DEPS:
        h.update(str(d.relative_to(ROOT)).encode() + b"\0")
        h.update(d.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:16]


def lib_build_id(path: Path = LIB) -> str | None:
    """The build id a built libmhmkc.so carries (its MHMKC_BUILD_ID= marker), read from the file without loading it."""
    if not path.exists():
        return None
    data = path.read_bytes()
    i = data.find(b"MHMKC_BUILD_ID=")
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + 15:j].decode(errors="replace")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _run(cmd, cwd=None):
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], cwd=cwd, check=True)


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found: libmhmkc.so cannot be built")


def _compile_lib(out: Path, bid: str, extra=(), tag: str = "main") -> None:
    """One hipcc per source, in parallel (the kernels file dominates), then one link."""
    from concurrent.futures import ThreadPoolExecutor

    obj_dir = ROOT / "build" / f"obj_{tag}"
    obj_dir.mkdir(parents=True, exist_ok=True)
    objs = [obj_dir / (src.name + ".o") for src in LIB_SOURCES]
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f'-DMHMKC_BUILD_ID="{bid}"', *extra]
    with ThreadPoolExecutor(max_workers=len(LIB_SOURCES)) as ex:
        list(ex.map(lambda so: _run([hipcc(), *flags, "-c", so[0], "-o", so[1]]), zip(LIB_SOURCES, objs)))
    tmp = out.with_suffix(".so.tmp")
    _run([hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", *objs, "-L/opt/rocm/lib", "-lrccl",
          "-Wl,-rpath,/opt/rocm/lib", "-o", tmp])
    tmp.replace(out)


def build_variant(name: str, defines) -> Path:
    """exp/libmhmkc_<name>.so with extra -D flags (performance A/B runs; MHMKC_LIB selects it). Its build id is the
    tree's with the flags' hash appended, so a variant never passes the check that the loaded library is the tree's."""
    out = ROOT / "exp" / f"libmhmkc_{name}.so"
    out.parent.mkdir(exist_ok=True)
    fh = hashlib.sha256("\0".join([ARCH, *defines]).encode()).hexdigest()[:8]
    _compile_lib(out, f"{source_build_id()}+{fh}", list(defines), tag=name)
    return out


def build_lib(force: bool = False) -> Path:
    bid = source_build_id()
    if force or _stale(LIB, LIB_DEPS) or lib_build_id() != bid:
        _compile_lib(LIB, bid)
    if lib_build_id() != bid:
        raise RuntimeError(f"{LIB} carries build id {lib_build_id()}, the sources make {bid}")
    return LIB


def build_synth(force: bool = False) -> Path:
    if force or _stale(SYNTH, SYNTH_DEPS):
        tmp = SYNTH.with_suffix(".so.tmp")
        _run(["gcc", "-O3", "-fPIC", "-shared", "-Wall", CSRC / "synth.c", "-lpthread", "-o", tmp])
        tmp.replace(SYNTH)
    return SYNTH


def build_oracle(force: bool = False) -> Path:
    odir = ROOT / "oracle"
    if force:
        _run(["make", "-C", odir, "clean"])
    _run(["make", "-s", "-C", odir])
    return ORACLE


def build_fill(force: bool = False) -> Path:
    if force or _stale(FILL, FILL_DEPS + [LIB]):
        FILL.parent.mkdir(parents=True, exist_ok=True)
        tmp = FILL.with_suffix(".tmp")
        _run(["g++", "-O2", "-std=c++17", "-pthread", "-I", ROOT / "include", FILL_DEPS[0], "-L", PKG, "-lmhmkc", "-lz",
              f"-Wl,-rpath,{PKG}", "-Wl,-rpath,$ORIGIN/../../mhm2_proxy_amd", "-o", tmp])
        tmp.replace(FILL)
    return FILL


def build_handoff(force: bool = False) -> Path:
    if force or _stale(HANDOFF, HANDOFF_DEPS + [LIB]):
        HANDOFF.parent.mkdir(parents=True, exist_ok=True)
        tmp = HANDOFF.with_suffix(".tmp")
        _run(["g++", "-O2", "-std=c++17", "-pthread", "-fPIC", "-shared", "-I", ROOT / "include", HANDOFF_DEPS[0], "-L",
              PKG, "-lmhmkc", "-lz", "-Wl,-rpath,$ORIGIN/../../mhm2_proxy_amd", "-o", tmp])
        tmp.replace(HANDOFF)
    return HANDOFF


def build_dbjg(force: bool = False) -> Path:
    if force or _stale(DBJG, DBJG_DEPS + [LIB]):
        DBJG.parent.mkdir(parents=True, exist_ok=True)
        tmp = DBJG.with_suffix(".tmp")
        _run(["g++", "-O2", "-std=c++17", "-pthread", "-fPIC", "-shared", "-I", ROOT / "include", DBJG_DEPS[0], "-L",
              PKG, "-lmhmkc", "-lz", "-Wl,-rpath,$ORIGIN/../../mhm2_proxy_amd", "-o", tmp])
        tmp.replace(DBJG)
    return DBJG


def build_all(force: bool = False) -> None:
    build_lib(force)
    build_synth(force)
    build_oracle(force)
    build_fill(force)
    build_handoff(force)
    build_dbjg(force)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":  # python -m mhm2_proxy_amd.build --variant NAME -DX=V ...
        print(build_variant(sys.argv[2], sys.argv[3:]))
    else:
        build_all(force="--force" in sys.argv)
