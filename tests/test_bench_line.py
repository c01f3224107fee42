"""The bench line's definitions, CPU only:
* RCCL's connection log lines parsed into per-pair transports, and the `rccl` record with its xgmi flag;
* line_problems(): every field's formula, on canned N = 1 / N > 1 lines, and on every bench line GPU runs
  of this round committed under profiles/r05/."""
import copy
import glob
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# RCCL INFO lines in the formats of the librccl.so torch ships (bench.py's comment lists them); the
# socket lines are what the one-GPU rehearsal (virtual hosts) logs, the P2P/IPC ones an xGMI node.
P2P_8 = [f"node:{100 + a}:{200 + a} [{a}] NCCL INFO Channel {c:02d}/0 : {a}[{a + 1:x}000] -> {b}[{b + 1:x}000] "
         f"via P2P/IPC comm 0x5566{a}0 nRanks 08"
         for a in range(8) for b in range(8) if a != b for c in range(2)]
SOCKET_2 = [
    "box:11:12 [0] NCCL INFO Channel 00/0 : 1[0] -> 0[0] [receive] via NET/Socket/0 comm 0x7f01 nRanks 02",
    "box:11:12 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0 comm 0x7f01 nRanks 02",
    "box:11:12 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[0] [send] via NET/Socket/0 comm 0x7f01 nRanks 02",
]
NOISE = [
    "box:11:12 [0] NCCL INFO Bootstrap : Using lo:127.0.0.1<0>",
    "box:11:12 [0] NCCL INFO Connected all rings, use ring PXN 0 GDR 1",
    "box:11:12 [0] NCCL INFO ncclCommInitRank comm 0x7f01 rank 0 nranks 2 cudaDev 0 busId 5000 - Init COMPLETE",
]


LIB = {"library": "/x/torch/lib/librccl.so", "version": "2.22.3", "version_code": 22203}


def _info(r, bus, n=8):
    return {"nranks": n, "rank": r, "device": r if bus else 0, "pci_bus_id": f"0000:{(r + 1) if bus else 5:02x}:00.0"}


def test_parse_p2p_socket_shm_and_noise():
    pairs = bench.parse_rccl_transports(P2P_8 + NOISE)
    assert len(pairs) == 56 and all(v == {"P2P/IPC"} for v in pairs.values())
    pairs = bench.parse_rccl_transports(SOCKET_2 + NOISE)
    assert pairs == {(1, 0): {"NET/Socket/0"}, (0, 1): {"NET/Socket/0"}}
    shm = "h:1:2 [3] NCCL INFO Channel 00 : 3[4c000] -> 2[3c000] via SHM/direct/direct comm 0x1 nRanks 04"
    direct = "h:1:2 [3] NCCL INFO Channel 01/0 : 3[4c000] -> 2[3c000] via P2P/direct pointer comm 0x1 nRanks 04"
    assert bench.parse_rccl_transports([shm, direct]) == {(3, 2): {"SHM/direct/direct", "P2P/direct pointer"}}
    # a communicator of another size (torch's own nccl group, a sub-communicator) is filtered out
    assert bench.parse_rccl_transports(SOCKET_2 + [shm], nranks=2) == bench.parse_rccl_transports(SOCKET_2)
    assert bench.parse_rccl_transports(NOISE) == {}


def test_transport_family():
    assert [bench.transport_family(t) for t in ("P2P/IPC", "P2P/IPC/read", "SHM/direct/direct", "NET/Socket/0",
                                                "NET/IB/0/GDRDMA", "what")] == ["P2P", "P2P", "SHM", "NET", "NET", "?"]


def test_record_xgmi_true_only_for_all_p2p_on_distinct_gpus():
    per_rank = [bench.parse_rccl_transports([ln for ln in P2P_8 if f"[{r}] NCCL" in ln], nranks=8) for r in range(8)]
    rec = bench.rccl_record([_info(r, True) for r in range(8)], per_rank, 8)
    assert rec["xgmi"] is True and rec["not_xgmi_because"] is None
    assert rec["nranks"] == 8 and rec["user_ranks"] == list(range(8)) and len(set(rec["pci_bus_ids"])) == 8
    assert rec["pairs_logged"] == 56 and rec["transports"] == {"P2P/IPC": 56}
    # one pair fell back to SHM: flagged, and named
    bad = copy.deepcopy(per_rank)
    bad[3][(3, 4)] = {"SHM/direct/direct"}
    rec = bench.rccl_record([_info(r, True) for r in range(8)], bad, 8)
    assert rec["xgmi"] is False and any("SHM" in w for w in rec["not_xgmi_because"])
    assert rec["pairs"]["3->4"] == "SHM/direct/direct"
    # a communicator that holds fewer ranks than launched
    rec = bench.rccl_record([_info(r, True, n=4) for r in range(8)], per_rank, 8)
    assert rec["xgmi"] is False and any("communicator sizes" in w for w in rec["not_xgmi_because"])
    # no log lines at all (NCCL_DEBUG overridden, or the log not written): never claimed as xGMI
    rec = bench.rccl_record([_info(r, True) for r in range(8)], [{} for _ in range(8)], 8)
    assert rec["xgmi"] is False and "no connection lines in the RCCL logs" in rec["not_xgmi_because"]


def test_record_one_gpu_rehearsal_is_net_socket_not_xgmi():
    """What the one-GPU `--gpus 2` rehearsal (CHR_BENCH_VIRTUAL_HOSTS=1) must show: 2 ranks, the socket
    transport, xgmi false."""
    per_rank = [bench.parse_rccl_transports(SOCKET_2, nranks=2), bench.parse_rccl_transports(SOCKET_2, nranks=2)]
    rec = bench.rccl_record([_info(0, False, 2), _info(1, False, 2)], per_rank, 2)
    assert rec["nranks"] == 2 and rec["user_ranks"] == [0, 1]
    assert rec["transports"] == {"NET/Socket/0": 2} and rec["xgmi"] is False
    assert any("NET" in w for w in rec["not_xgmi_because"])
    assert any("1 distinct PCI devices" in w for w in rec["not_xgmi_because"])


def test_rccl_log_env_is_per_rank_file(tmp_path):
    env = bench.rccl_log_env(3, str(tmp_path / "logs"))
    assert env["NCCL_DEBUG"] == "INFO" and env["NCCL_DEBUG_SUBSYS"] == "INIT"
    assert env["NCCL_DEBUG_FILE"].startswith(str(tmp_path / "logs" / "rccl.rank3."))
    (tmp_path / "logs" / "rccl.rank3.77.log").write_text("\n".join(SOCKET_2))
    (tmp_path / "logs" / "rccl.rank1.78.log").write_text("x")
    assert bench.read_rccl_logs(str(tmp_path / "logs"), 3) == SOCKET_2
    assert bench.read_rccl_logs(str(tmp_path / "nowhere"), 3) == []


def test_stale_rccl_log_is_ignored(tmp_path):
    """a file an earlier run left in the log directory (another pid: P2P lines that would make
    the record claim xGMI) is not read into this run's pairs; only this process's own file is."""
    logs = tmp_path / "logs"
    logs.mkdir()
    (logs / "rccl.rank0.111.log").write_text("\n".join(ln for ln in P2P_8 if "[0] NCCL" in ln))  # stale
    (logs / "rccl.rank0.222.log").write_text("\n".join(SOCKET_2))                               # this run
    got = bench.parse_rccl_transports(bench.read_rccl_logs(str(logs), 0, 222), nranks=2)
    assert got == bench.parse_rccl_transports(SOCKET_2, nranks=2)
    assert bench.read_rccl_logs(str(logs), 0, 333) == []


def test_rccl_library_names_the_loaded_copy():
    """rccl_library() on this process: the path comes from /proc/self/maps only (None when no librccl is loaded,
    as in a CPU test that has not imported torch's RCCL), never from a fresh dlopen."""
    rec = bench.rccl_library()
    assert set(rec) == {"library", "version", "version_code"}
    if rec["library"] is not None:
        assert "librccl" in os.path.basename(rec["library"])
        assert rec["version_code"] is None or rec["version_code"] > 20000
    # the record carries rank 0's library and whether every rank agrees
    recs = [bench.rccl_record([_info(r, True) for r in range(2)], [{}, {}], 2, libs)
            for libs in ([LIB, LIB], [LIB, dict(LIB, version="2.27.3")])]
    assert recs[0]["version"] == "2.22.3" and recs[0]["same_on_all_ranks"] is True
    assert recs[1]["same_on_all_ranks"] is False


def _n1_line():
    by, span = 3 * 4 * bench.C2_ELEMS, 0.0302
    ach = by / (span * 1e-3) / 1e9
    return {"metric": bench.METRIC, "value": round(ach, 2), "unit": "GB/s", "n_gpus": 1, "steps": 20, "warmup": 5,
            "ms_per_step": span, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic", "config": {"workload": "C2"},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(ach / 8000, 4), "traffic": None, "traffic_stale": "x",
                         "algorithmic_bytes_per_launch": by, "event_span_ms_per_launch": span},
            "cpu_baseline": {"value": 69.0, "unit": "GB/s", "cores": 1, "kind": "reference", "sample": "s"},
            "definitions": bench.LINE_DEFINITIONS_N1}


def _nn_line(n=8):
    count, ms = 1 << 28, 5.0
    S = 4 * count
    algbw = S / (ms * 1e-3) / 1e9
    return {"metric": bench.METRIC, "value": round(n * algbw, 2), "unit": "GB/s", "n_gpus": n, "steps": 20,
            "warmup": 5, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {"workload": "C4", "k": 4, "b": 4, "count": count, "schedule": "auto -> flat, 4 slices",
                       "slices": 4, "overlap": True},
            "algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * 2 * (n - 1) / n, 2),
            "aggregate_GBps": round(n * algbw, 2), "definitions": bench.LINE_DEFINITIONS_NN,
            "roofline": {"traffic": 123, "traffic_source": "pmc"},
            "rccl": bench.rccl_record([_info(r, True) for r in range(n)],
                                      [bench.parse_rccl_transports(P2P_8, nranks=8)] * n, n, [LIB] * n),
            "cpu_baseline": {"value": 3.0, "unit": "GB/s", "cores": n, "kind": "reference", "sample": "s"},
            "result_check": {"ranks_bit_identical": True, "within_tolerance": True, "violations": 0},
            "compare": {"c5_allreduce_bf16_k4_b4_1GiB": {"algbw_GBps": 1, "schedule": "flat", "slices": 4,
                                                         "overlap": True}}}


def test_canned_lines_pass():
    assert bench.line_problems(_n1_line()) == []
    assert bench.line_problems(_nn_line()) == []


@pytest.mark.parametrize("mutate, problem", [
    (lambda l: l.__setitem__("value", l["value"] * 8), "value"),
    (lambda l: l.__setitem__("busbw_GBps", l["algbw_GBps"]), "busbw"),
    (lambda l: l.__setitem__("algbw_GBps", l["value"]), "algbw"),
    (lambda l: l["config"].pop("slices"), "config.slices"),
    (lambda l: l.pop("rccl"), "rccl"),
    (lambda l: l["rccl"].__setitem__("not_xgmi_because", ["x"]), "xgmi true"),
    (lambda l: l["rccl"].pop("version"), "rccl.version"),
    (lambda l: l["rccl"].pop("library"), "rccl.library"),
    (lambda l: l["rccl"].__setitem__("same_on_all_ranks", False), "rccl.same_on_all_ranks"),
    (lambda l: l["roofline"].update(traffic=None), "traffic"),
    (lambda l: l["compare"]["c5_allreduce_bf16_k4_b4_1GiB"].pop("overlap"), "c5.overlap"),
    (lambda l: l["compare"]["c5_allreduce_bf16_k4_b4_1GiB"].update(slices=1), "overlapped depth"),
    (lambda l: l["compare"]["c5_allreduce_bf16_k4_b4_1GiB"].update(
        result_check={"ranks_bit_identical": False, "within_tolerance": True}), "c5 result_check"),
    (lambda l: l["result_check"].update(ranks_bit_identical=False), "result_check failed"),
])
def test_nn_line_definitions_are_enforced(mutate, problem):
    line = _nn_line()
    mutate(line)
    assert any(problem in p for p in bench.line_problems(line)), bench.line_problems(line)


def test_n1_line_definitions_are_enforced():
    line = _n1_line()
    line["roofline"]["avg_kernel_ms"] = line["roofline"].pop("event_span_ms_per_launch")
    assert any("avg_kernel_ms" in p for p in bench.line_problems(line))
    line = _n1_line()
    line["roofline"]["achieved"] *= 1.1
    assert any("achieved" in p for p in bench.line_problems(line))


def test_committed_round5_lines_meet_the_definitions():
    """Every bench line a GPU run of this round committed (profiles/r05/**/bench*.json) obeys the same
    definitions."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r05", "**", "bench*.json"), recursive=True))
    checked = 0
    for f in files:
        try:
            with open(f) as fh:
                line = json.loads(fh.read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        if "metric" not in line:
            continue
        assert bench.line_problems(line, rccl_library=False) == [], f
        checked += 1
    if not files:
        pytest.skip("no round-5 bench lines committed yet")


@pytest.mark.parametrize("n, k, b, want", [(2, 2, 2, "reduce_f32_sum_m1_oop_128MiB"), (4, 4, 4, "reduce_f32_sum_m3_oop_64MiB"),
                                           (8, 4, 4, "tree_f32_sum_8leaves_64MiB")])
@pytest.mark.parametrize("slices", [1, 4, 8])
def test_roofline_binds_the_kernel_the_plan_launches(n, k, b, want, slices):
    """The N>1 line's roofline.traffic comes from the PMC entry of the kernel the metric's plan launches: the N = 2 / N = 4
    lines' one-node geometries compile each piece's expression to ONE fold (k_reduce_vec out of place), C4's to 8-leaf
    trees -- read off the plan (chr_plan_describe, host only), not assumed from N."""
    import chiara_amd as ca

    plan = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, n, 0, k, b, 1 << 28, slices, ca.SCHEDULE_FLAT))
    (key, sym), why = bench.reduction_pmc(plan)
    assert why is None and key == want
    assert ("k_reduce_tree<0, 0, 8," in sym) == (n == 8)
