"""ctypes bindings of libmhmkc.so (include/mhmkc.h) and libmhmkc_synth.so (include/mhmkc_synth.h).

There is no fallback: if the HIP library is missing, loading raises. The product path never touches
oracle/ (the CPU checker lives there and is loaded only by tests and the bench's cpu_baseline leg).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import os

PKG = Path(__file__).resolve().parent
# MHMKC_LIB selects another build of the same library (performance experiments, tools/ab.sh)
LIB_PATH = Path(os.environ["MHMKC_LIB"]) if os.environ.get("MHMKC_LIB") else PKG / "libmhmkc.so"
SYNTH_PATH = PKG / "libmhmkc_synth.so"

MHMKC_COMM_ID_BYTES = 128

ERRORS = {
    0: "MHMKC_OK",
    -1: "MHMKC_EINVAL",
    -2: "MHMKC_ENOMEM",
    -3: "MHMKC_EHIP",
    -4: "MHMKC_ERCCL",
    -5: "MHMKC_ESTATE",
    -6: "MHMKC_EBADCHAR",
    -7: "MHMKC_EUNSUPPORTED",
    -8: "MHMKC_ETRANSPORT",
}

MHMKC_OWNER_HASH = 0
MHMKC_OWNER_MINIMIZER = 1

STAGES = ["tileidx", "extract_hist", "extract_scatter", "exchange", "part_hist", "part_scatter", "count", "other"]

# every symbol include/mhmkc.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = [
    "mhmkc_config_init", "mhmkc_create", "mhmkc_destroy", "mhmkc_comm_id", "mhmkc_add_reads",
    "mhmkc_add_reads_device", "mhmkc_add_seqs", "mhmkc_add_ctgs", "mhmkc_finish", "mhmkc_fetch", "mhmkc_fetch_ordered",
    "mhmkc_fetch_ordered_range", "mhmkc_fetch_map_range", "mhmkc_host_alloc", "mhmkc_host_free",
    "mhmkc_device_output",
    "mhmkc_get_stats", "mhmkc_reset", "mhmkc_set_profiling", "mhmkc_last_error", "mhmkc_abi_version",
    "mhmkc_build_id",
    "mhmkc_add_fastq", "mhmkc_add_fastq_device", "mhmkc_add_fastq_pairs", "mhmkc_add_fastq_pairs_device",
    "mhmkc_add_fastq_file", "mhmkc_add_fastq_pairs_file",
    "mhmkc_fastq_packed", "mhmkc_fastq_fetch",
    "mhmkc_wait_stream", "mhmkc_set_dmin_thres", "mhmkc_set_transport", "mhmkc_minimizer_hashes",
]
SYNTH_SYMBOLS = ["mhmkc_synth_config_init", "mhmkc_synth_genome", "mhmkc_synth_reads"]
# the test-only entry point (include/mhmkc_debug.h)
DEBUG_SYMBOLS = ["mhmkc_debug_nib_pack", "mhmkc_debug_reset", "mhmkc_debug_set"]


class MhmkcConfig(C.Structure):
    _fields_ = [
        ("k", C.c_int32),
        ("n_longs", C.c_int32),
        ("qual_offset", C.c_int32),
        ("qual_cutoff", C.c_int32),
        ("dmin_thres", C.c_int32),
        ("dyn_min_depth", C.c_double),
        ("device", C.c_int32),
        ("rank", C.c_int32),
        ("n_ranks", C.c_int32),
        ("comm_id", C.c_void_p),
        ("stream", C.c_void_p),
        ("output_owner", C.c_int32),
        ("minimizer_len", C.c_int32),
    ]


class MhmkcStats(C.Structure):
    _fields_ = [
        ("reads", C.c_uint64),
        ("bases", C.c_uint64),
        ("occurrences", C.c_uint64),
        ("owned_records", C.c_uint64),
        ("distinct", C.c_uint64),
        ("purged", C.c_uint64),
        ("n_out", C.c_uint64),
        ("dropped", C.c_uint64),
        ("count_sum", C.c_uint64),
        ("overflow_sweeps", C.c_uint64),
        ("max_bucket", C.c_uint64),
        ("fine_buckets", C.c_uint64),
        ("bytes_sent", C.c_uint64),
        ("exact_reruns", C.c_uint64),
        ("ctg_kmers", C.c_uint64),
        ("coarse_record_bytes", C.c_uint64),
        ("fine_record_bytes", C.c_uint64),
        ("distinct_estimate", C.c_uint64),
        ("ms_total", C.c_double),
        ("ms_kernel", C.c_double * 8),
        ("launches", C.c_uint64 * 8),
        ("bytes_recv", C.c_uint64),
        ("handoff_sent", C.c_uint64),
        ("handoff_recv", C.c_uint64),
        ("h2d_bytes", C.c_uint64),
        ("h2d_chunks", C.c_uint64),
        ("slabs", C.c_uint64),
        ("ms_h2d", C.c_double),
        ("lds_misses", C.c_uint64),
        ("lds_ext_adds", C.c_uint64),
        ("fq_pairs", C.c_uint64),
        ("fq_merged", C.c_uint64),
        ("fq_ambiguous", C.c_uint64),
        ("fq_overlap_bases", C.c_uint64),
        ("table_slots", C.c_uint64),
        ("fq_file_blocks", C.c_uint64),
        ("smer_count", C.c_uint64),
        ("smer_words", C.c_uint64),
        ("xchg_rounds", C.c_uint64),
        ("ms_xchg", C.c_double),
        ("ms_xchg_exposed", C.c_double),
        ("finish_passes", C.c_uint64),
        ("out_reruns", C.c_uint64),
        ("device_bytes", C.c_uint64),
        ("device_bytes_peak", C.c_uint64),
        ("inc_rounds", C.c_uint64),
        ("inc_fallbacks", C.c_uint64),
        ("ms_finish_tail", C.c_double),
        ("inc_redone_coarse", C.c_uint64),
        ("inc_slack", C.c_double),
        ("ms_h2d_pack", C.c_double),
        ("ms_h2d_wait", C.c_double),
        ("ms_h2d_rounds", C.c_double),
        ("h2d_raw_chunks", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ("ms_kernel", "launches")}
        d["ms_kernel"] = {STAGES[i]: self.ms_kernel[i] for i in range(8)}
        d["launches"] = {STAGES[i]: int(self.launches[i]) for i in range(8)}
        return d


# mhmkc_transport (host-staged exchange between ranks)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p, C.POINTER(C.c_uint64))


class MhmkcTransport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


class SynthConfig(C.Structure):
    _fields_ = [
        ("genome_len", C.c_uint64),
        ("read_len", C.c_uint32),
        ("seed", C.c_uint64),
        ("sub_rate", C.c_double),
        ("n_rate", C.c_double),
        ("lowq_rate", C.c_double),
        ("subq_prob", C.c_double),
    ]


_lib = None
_synth = None


def _bind_torch_runtime() -> None:
    """Load torch's HIP runtime before libmhmkc.so when torch is importable.

    torch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1 / librccl.so.1 with the same SONAMEs as
    /opt/rocm; whichever copy is loaded first serves the whole process. libmhmkc.so works on either,
    torch only on its own, so torch goes first (measured: tools/probe_runtime.py). MHMKC_NO_TORCH=1
    skips this (pure C/C++ hosts never load torch).
    """
    import os

    if os.environ.get("MHMKC_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401  (loads libtorch_hip -> torch/lib/libamdhip64.so.7)
    except Exception:
        pass


def debug_set(knob: str, value: int) -> None:
    """A test-only switch of the library (include/mhmkc_debug.h: exact layouts, tiny tables, ...); tests only."""
    if lib().mhmkc_debug_set(knob.encode(), int(value)) != 0:
        raise ValueError(f"unknown debug knob {knob!r}")


def debug_reset() -> None:
    if _lib is not None:
        _lib.mhmkc_debug_reset()


def lib() -> C.CDLL:
    """Load libmhmkc.so (raises if it has not been built: no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} is missing: run `python -m mhm2_proxy_amd.build` "
                          "(the HIP extension is required; there is no CPU fallback)")
    _bind_torch_runtime()
    L = C.CDLL(str(LIB_PATH))
    P, U64, I32, VP = C.POINTER, C.c_uint64, C.c_int, C.c_void_p
    L.mhmkc_config_init.argtypes = [P(MhmkcConfig)]
    L.mhmkc_create.argtypes = [P(VP), P(MhmkcConfig)]
    L.mhmkc_destroy.argtypes = [VP]
    L.mhmkc_destroy.restype = None
    L.mhmkc_comm_id.argtypes = [VP]
    L.mhmkc_add_reads.argtypes = [VP, VP, VP, U64]
    L.mhmkc_add_reads_device.argtypes = [VP, VP, VP, U64, U64]
    L.mhmkc_add_seqs.argtypes = [VP, C.c_char_p, VP, U64, C.c_uint16]
    L.mhmkc_add_ctgs.argtypes = [VP, C.c_char_p, VP, VP, U64]
    L.mhmkc_add_fastq.argtypes = [VP, C.c_char_p, U64]
    L.mhmkc_add_fastq_device.argtypes = [VP, VP, U64]
    L.mhmkc_add_fastq_pairs.argtypes = [VP, C.c_char_p, U64]
    L.mhmkc_add_fastq_pairs_device.argtypes = [VP, VP, U64]
    L.mhmkc_add_fastq_file.argtypes = [VP, C.c_char_p]
    L.mhmkc_add_fastq_pairs_file.argtypes = [VP, C.c_char_p]
    L.mhmkc_fastq_packed.argtypes = [VP, P(VP), P(VP), P(U64), P(U64)]
    L.mhmkc_fastq_fetch.argtypes = [VP, VP, VP]
    L.mhmkc_finish.argtypes = [VP, P(U64)]
    L.mhmkc_fetch.argtypes = [VP, VP, VP, VP, VP]
    L.mhmkc_fetch_ordered.argtypes = [VP, VP, VP, VP, VP]
    L.mhmkc_fetch_ordered_range.argtypes = [VP, U64, U64, VP, VP, VP, VP]
    L.mhmkc_fetch_map_range.argtypes = [VP, U64, U64, U64, VP, VP, VP, VP, VP, VP]
    L.mhmkc_host_alloc.argtypes = [U64]
    L.mhmkc_host_alloc.restype = VP
    L.mhmkc_host_free.argtypes = [VP]
    L.mhmkc_host_free.restype = None
    L.mhmkc_debug_set.argtypes = [C.c_char_p, C.c_int64]
    L.mhmkc_debug_reset.argtypes = []
    L.mhmkc_debug_reset.restype = None
    L.mhmkc_debug_nib_pack.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_int]
    L.mhmkc_device_output.argtypes = [VP, P(VP), P(VP), P(VP), P(VP), P(U64)]
    L.mhmkc_get_stats.argtypes = [VP, P(MhmkcStats)]
    L.mhmkc_reset.argtypes = [VP]
    L.mhmkc_set_profiling.argtypes = [VP, I32]
    L.mhmkc_last_error.argtypes = [VP]
    L.mhmkc_last_error.restype = C.c_char_p
    L.mhmkc_abi_version.argtypes = []
    L.mhmkc_build_id.argtypes = []
    L.mhmkc_build_id.restype = C.c_char_p
    L.mhmkc_wait_stream.argtypes = [VP, VP]
    L.mhmkc_set_dmin_thres.argtypes = [VP, C.c_int32]
    L.mhmkc_set_transport.argtypes = [VP, P(MhmkcTransport)]
    L.mhmkc_minimizer_hashes.argtypes = [VP, VP, U64, C.c_int32, C.c_int32, VP]
    _lib = L
    return L


def build_id() -> str:
    """The build id compiled into the loaded libmhmkc.so (include/mhmkc.h mhmkc_build_id)."""
    return lib().mhmkc_build_id().decode()


def synth() -> C.CDLL:
    global _synth
    if _synth is not None:
        return _synth
    if not SYNTH_PATH.exists():
        raise ImportError(f"{SYNTH_PATH} is missing: run `python -m mhm2_proxy_amd.build`")
    S = C.CDLL(str(SYNTH_PATH))
    S.mhmkc_synth_config_init.argtypes = [C.POINTER(SynthConfig), C.c_uint64, C.c_uint32, C.c_uint64]
    S.mhmkc_synth_genome.argtypes = [C.POINTER(SynthConfig), C.c_void_p]
    S.mhmkc_synth_reads.argtypes = [C.POINTER(SynthConfig), C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                    C.c_void_p, C.c_int]
    _synth = S
    return S


class MhmkcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def check(code: int, handle=None) -> None:
    if code != 0:
        msg = lib().mhmkc_last_error(handle)
        raise MhmkcError(code, msg.decode() if msg else "")
