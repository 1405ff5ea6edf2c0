"""mhm2_proxy_amd — MI355X-native k-mer counting stage (kcount) for the MetaHipMer2 contigging path.

Drop-in for the reference's kcount hot path (ajpowelsnl/mhm2_proxy src/kcount/): the C ABI is
include/mhmkc.h (libmhmkc.so, HIP kernels for gfx950), include/mhmkc_kcount.hpp rebuilds the reference
C++ shapes on top of it, and this package mirrors them in Python (mhm2_proxy_amd.kcount).
"""
from .kcount import (  # noqa: F401
    KmerCounter,
    KmerCounts,
    KmerDHT,
    KmerTable,
    PackedReads,
    SharedGpuCounter,
    TorchDistTransport,
    analyze_kmers,
    comm_id,
    get_kmer_target_rank,
    kmer_from_string,
    kmer_to_string,
    keys_to_strings,
    n_longs_for,
    synth_genome,
    synth_reads,
)
from ._native import MHMKC_OWNER_HASH, MHMKC_OWNER_MINIMIZER, MhmkcError  # noqa: F401

__all__ = [
    "KmerCounter", "KmerCounts", "KmerDHT", "KmerTable", "PackedReads", "analyze_kmers", "comm_id",
    "get_kmer_target_rank", "kmer_from_string", "kmer_to_string", "keys_to_strings", "n_longs_for",
    "synth_genome", "synth_reads", "MhmkcError", "TorchDistTransport", "MHMKC_OWNER_HASH", "MHMKC_OWNER_MINIMIZER",
    "SharedGpuCounter",
]
