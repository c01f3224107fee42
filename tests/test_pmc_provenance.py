"""roofline.traffic is bound to the kernel it was measured on: bench.py reports a
PMC figure only while the kernel symbol and the hash of its sources match the committed entry."""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import pmc_provenance as pp  # noqa: E402

KEY = "reduce_f32_sum_m1_64MiB"
SYM = "void chr::k_reduce_vec<0, 0, 1, 4, true, true, 64>(chr::VecArgs)"


def _tree(tmp_path):
    root = tmp_path / "repo"
    for rel in pp.KERNEL_SOURCES[KEY]:
        (root / rel).parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(REPO, rel), root / rel)
    (root / "profiles").mkdir()
    entry = {"hbm_bytes_per_launch": 201356288.0, "kernel_symbol": SYM,
             "sources_sha256_16": pp.sources_hash(KEY, str(root))}
    (root / "profiles" / "pmc_latest.json").write_text(json.dumps({"kernels": {KEY: entry}}))
    return root, entry


def test_matching_entry_reports_traffic(tmp_path):
    root, entry = _tree(tmp_path)
    assert pp.current_traffic(entry, KEY, SYM, str(root)) == (201356288.0, None)


def test_one_flipped_source_byte_makes_traffic_null(tmp_path):
    root, entry = _tree(tmp_path)
    src = root / pp.KERNEL_SOURCES[KEY][0]
    data = bytearray(src.read_bytes())
    data[len(data) // 2] ^= 0x01
    src.write_bytes(bytes(data))
    traffic, why = pp.current_traffic(entry, KEY, SYM, str(root))
    assert traffic is None and "changed" in why


def test_other_kernel_symbol_makes_traffic_null(tmp_path):
    root, entry = _tree(tmp_path)
    traffic, why = pp.current_traffic(entry, KEY, SYM.replace("1, 4", "1, 2"), str(root))
    assert traffic is None and "measured on" in why


def test_bench_reads_through_provenance(tmp_path):
    import bench

    root, _ = _tree(tmp_path)
    assert bench.pmc_traffic(KEY, bench.C2_KERNEL_SYMBOL, str(root)) == (201356288.0, None)
    src = root / pp.KERNEL_SOURCES[KEY][1]
    src.write_bytes(src.read_bytes() + b" ")
    traffic, why = bench.pmc_traffic(KEY, bench.C2_KERNEL_SYMBOL, str(root))
    assert traffic is None and why


def test_every_reduction_shape_has_its_entry():
    """Every PMC entry a bench line can bind (bench.TREE_PMC, bench.VEC_OOP_PMC; chosen off the plan by
    bench.reduction_pmc) has sources registered, and names the streaming instantiation the library ships: trees at
    reduce_tree.hpp's tree_u (U = 1 / 2 / 4) with the ACC0 slot, folds at reduce_vec.hpp's vec_u_nt (U = 4 / 2) with
    theirs.  Whether the committed figures are current is the bench line's own `traffic_stale`."""
    import bench

    for nl, (key, sym) in bench.TREE_PMC.items():
        assert key in pp.KERNEL_SOURCES
        if nl == 2:  # a streaming 2-leaf tree is one out-of-place fold on the bucket kernel (reduce_tree.hip)
            assert sym == bench.VEC_OOP_PMC[1][1]
            continue
        assert f"k_reduce_tree<0, 0, {nl}, {dict([(8, 1), (4, 2)])[nl]}, true, 64, true>" in sym
    for m, (key, sym) in bench.VEC_OOP_PMC.items():
        assert key in pp.KERNEL_SOURCES
        assert f"k_reduce_vec<0, 0, {m}, {dict([(1, 4), (3, 2)])[m]}, true, true, 64>" in sym
