"""Provenance of the PMC traffic figures in profiles/pmc_latest.json.

A `roofline.traffic` figure is the HBM bytes per launch that rocprofv3's FETCH_SIZE / WRITE_SIZE
passes measured for one kernel instantiation built from one revision of its sources.  Each entry
records the kernel symbol the counters were collected on and a hash of the sources that define it;
bench.py reports the figure only while both still match (else traffic = null plus a
`traffic_stale` note), so a kernel change cannot leave a stale ratio in a BENCH line.
"""
import hashlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = "configurable-hierarchical-allreduce-algorithms_amd/csrc"

# pmc_latest.json key -> the sources its kernel is compiled from (repo-relative)
KERNEL_SOURCES = {
    "reduce_f32_sum_m1_64MiB": [f"{CSRC}/reduce_vec.hpp", f"{CSRC}/reduce_common.hpp", f"{CSRC}/reduce_kernels.hip",
                                f"{CSRC}/chr_internal.hpp"],
    "tree_f32_sum_8leaves_64MiB": [f"{CSRC}/reduce_tree.hpp", f"{CSRC}/reduce_common.hpp", f"{CSRC}/reduce_tree.hip",
                                   f"{CSRC}/chr_internal.hpp"],
}
# the 4-leaf tree (the tree API; no flat plan of a bench line launches it) comes from the same sources; a streaming
# 2-leaf tree runs on the bucket kernel, routed there by reduce_tree.hip (round 6)
KERNEL_SOURCES["tree_f32_sum_4leaves_64MiB"] = KERNEL_SOURCES["tree_f32_sum_8leaves_64MiB"]
KERNEL_SOURCES["tree_f32_sum_2leaves_64MiB"] = KERNEL_SOURCES["reduce_f32_sum_m1_64MiB"] + [f"{CSRC}/reduce_tree.hip"]
# the N = 2 / N = 4 lines' reductions: one fold per piece, out of place (recv = send (op) stage...), on the bucket
# kernel (schedule.cpp tree_program: a single fold is one k_reduce_vec launch)
KERNEL_SOURCES["reduce_f32_sum_m1_oop_128MiB"] = KERNEL_SOURCES["reduce_f32_sum_m1_64MiB"]
KERNEL_SOURCES["reduce_f32_sum_m3_oop_64MiB"] = KERNEL_SOURCES["reduce_f32_sum_m1_64MiB"]


def sources_hash(key, root=REPO):
    """sha256 over (path, contents) of the key's sources, first 16 hex digits."""
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES[key]:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def current_traffic(entry, key, symbol, root=REPO):
    """(hbm_bytes_per_launch, None) if the entry was measured on `symbol` built from the sources as
    they are now under `root`; else (None, reason)."""
    if entry is None:
        return None, f"no PMC entry for {key}"
    if entry.get("kernel_symbol") != symbol:
        return None, f"PMC entry measured on {entry.get('kernel_symbol')!r}, this run launches {symbol!r}"
    try:
        now = sources_hash(key, root)
    except OSError as e:
        return None, f"sources unreadable: {e}"
    if entry.get("sources_sha256_16") != now:
        return None, (f"kernel sources changed since the PMC passes (hash {entry.get('sources_sha256_16')} "
                      f"measured, {now} now): re-run tools/gpu.sh pmc")
    return entry.get("hbm_bytes_per_launch"), None
