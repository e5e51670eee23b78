"""The bench's cpu_baseline legs run the oracle on the host (bench.py main / main_partial):
both must run to completion on CPU, small and fast (no GPU)."""
import oracle_py


def test_scaled_bench_sample_runs():
    nodes, secs = oracle_py.bench_sample(512, lists=5, max_nodes=64, min_seconds=0.05)
    assert nodes > 0 and secs > 0


def test_partial_cpu_leg_runs():
    ora = oracle_py.PartialOracle(4096, v=32, rd_seed=7, view_seed=5, init_t0=8, init_seed=11, drop_pct=5,
                                  drop_from=0, drop_to=1 << 20, drop_seed=42)
    for _ in range(3):
        ora.tick()
    sent, recv = ora.last_msgcount()
    assert sent.sum() > 0 and recv.sum() > 0


def test_hour_run_reads_committed_segments():
    """bench.py's cpu_baseline.hour_run: the committed CPU-hour segments summed per tick (no re-run)."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    hr = bench.hour_run()
    assert hr is not None and hr["n"] == 13722 and hr["cores"] == 1
    assert hr["seconds"] > 0 and hr["value"] > 0 and "cpu_hour_seg" in hr["source"]
