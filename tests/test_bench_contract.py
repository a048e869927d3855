"""CPU checks of bench.py's workload contract: the default is the metric's configuration
(C3 shard), its paged capacities fit the documents-per-CU budget with a full-capacity tier
behind them, and the recorded evidence it quotes (PMC traffic, CPU calibration) matches it."""
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def _configs():
    return json.load(open(os.path.join(REPO, "bench", "configs.json")))


def test_default_workload_is_the_metric_config(bench, monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py"])
    args = bench.parse()
    assert args.config == "c3" and args.gpus == 1
    cfg = _configs()["c3"]
    assert cfg["docs"] == 100000 and cfg["ops"] == 10000
    # the metric's fixed 100k-document job: all of it on one GPU, 12.5k-document shards on 8
    assert bench.shard_plan(args, cfg, 1, 0) == (100000, 0, 100000, "strong")
    assert bench.shard_plan(args, cfg, 8, 3) == (12500, 37500, 100000, "strong")
    plans = [bench.shard_plan(args, cfg, 3, r) for r in range(3)]
    assert sum(p[0] for p in plans) == 100000 and [p[1] for p in plans] == [0, 33334, 66667]
    # --docs D: D per rank (weak scaling); --shard r: one shard of the 8-way split on one GPU
    monkeypatch.setattr("sys.argv", ["bench.py", "--docs", "2048"])
    assert bench.shard_plan(bench.parse(), cfg, 4, 2) == (2048, 4096, 8192, "weak")
    monkeypatch.setattr("sys.argv", ["bench.py", "--shard", "7"])
    assert bench.shard_plan(bench.parse(), cfg, 1, 0) == (12500, 87500, 12500, "weak")


def test_gpurun_ignore_keeps_transpiled_reference_home():
    """The transpiled reference (oracle/_ref, built in this container) must never be pushed to
    the GPU box: tar's exclude patterns as gpurun applies them leave none of it in the tree."""
    import subprocess
    ref = os.path.join(REPO, "oracle", "_ref")
    if not os.path.isdir(ref):
        pytest.skip("oracle/_ref not built here")
    out = subprocess.run(["tar", "--exclude=./.git", "--exclude-from=.gpurunignore", "-cf", "-",
                          "./oracle"], cwd=REPO, capture_output=True, check=True).stdout
    names = subprocess.run(["tar", "-t"], input=out, capture_output=True, check=True).stdout.decode()
    assert "oracle/ref_harness.mjs" in names
    assert not [n for n in names.split() if "oracle/_ref" in n]


def test_paged_capacities_tight_then_full(bench):
    cfg = _configs()["c3"]
    caps = bench.capacities(cfg)
    # tight LDS tier from measured peaks over all 100k C3 documents (183 / 208 / 173); the
    # HBM arrays and the full tier take any document that outgrows it (library hand-over)
    assert (caps["lds_page_capacity"], caps["lds_unsettled_capacity"], caps["lds_page_heap_capacity"]) == (192, 220, 192)
    for k in ("page_capacity", "unsettled_capacity", "page_heap_capacity"):
        assert caps[k] >= caps["lds_" + k]
    assert "lds_page_capacity" not in bench.capacities(cfg, tight=False)
    # the deep-lag config: a packed tight tier above the measured peaks over 4096 documents
    # (208 / 1810 / 841) that fits 3 documents per CU; the full tier behind it larger still
    c4 = bench.capacities(_configs()["c4"])
    assert all(c4["lds_" + k] >= peak for k, peak in
               (("page_capacity", 208), ("unsettled_capacity", 1810), ("page_heap_capacity", 841)))
    for k in ("page_capacity", "unsettled_capacity", "page_heap_capacity"):
        assert c4[k] >= c4["lds_" + k]


def test_recorded_traffic_matches_default_workload():
    pm = json.load(open(os.path.join(REPO, "profiles", "pmc_summary.json")))
    e = pm["c3"]
    assert e["docs"] == 100000 and e["ops"] == 10000 and e["hbm_bytes_per_launch"] > 0
    src = os.path.join(REPO, e["note"].split("source ")[-1])
    assert os.path.exists(src)


def test_cpu_calibration_recorded():
    import bench
    cal = json.load(open(bench.CALIBRATION))
    for name in ("c2", "c3"):
        c = cal[name]
        assert c["threads"] == 1 and c["ops"] > 0 and c["docs"] >= 16
        for sfx in ("", "_nocb"):
            r = c["ratio_port_over_reference" + sfx]
            assert r > 0 and abs(c["port_ops_per_s"] / c["reference" + sfx + "_ops_per_s"] - r) < 0.01 * r
        # the reference without a callback is at least as fast as with the position-recording one
        assert c["reference_nocb_ops_per_s"] >= 0.95 * c["reference_ops_per_s"]


@pytest.mark.parametrize("config,runner", [("c2", "run_replay"), ("c3", "run_replay"), ("c4", "run_replay"),
                                           ("c5", "run_c5"), ("live", "run_live"), ("c3skew", "run_skew")])
def test_every_config_reaches_its_runner(bench, monkeypatch, config, runner):
    """`bench.py --config X` calls X's own runner (round 4 lost the C5 branch behind the
    c3skew one: `--config c5` replayed C3 streams under a C5 label)."""
    import bench_skew
    calls = []
    for name in ("run_replay", "run_c5", "run_live"):
        monkeypatch.setattr(bench, name, lambda *a, _n=name, **k: calls.append((_n, a)))
    monkeypatch.setattr(bench_skew, "run_skew", lambda *a, **k: calls.append(("run_skew", a)))
    monkeypatch.setattr("sys.argv", ["bench.py", "--config", config])
    bench.main()
    assert [c[0] for c in calls] == [runner]
    if runner in ("run_replay", "run_c5", "run_skew"):
        cfg = calls[0][1][1]
        assert cfg == _configs()[config]


def test_unknown_config_is_refused(bench, monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py", "--config", "c9"])
    with pytest.raises(SystemExit):
        bench.main()
