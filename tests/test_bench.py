"""Host logic of bench.py that shapes the driver's line (no GPU): the clock
settling loop's stopping rules, and the algorithmic work model."""
import bench


def _fake_chunks(durations):
    it = iter(durations)
    clock = [0.0]

    def now():
        return clock[0]

    def run_chunk():
        clock[0] += next(it)
    return now, run_chunk


def test_settle_stops_when_two_chunks_agree(monkeypatch):
    # a ramp 170 -> 147 us per iteration in 20-iteration chunks: stops at the
    # first pair within 1% once 50 ms have passed
    per_it = [170, 165, 160, 156, 152, 149, 147.5, 147.2, 147.1, 147.0] + [147.0] * 40
    now, run_chunk = _fake_chunks([x * 20e-6 for x in per_it])
    monkeypatch.setattr(bench.time, "perf_counter", now)
    r = bench.settle_clocks(run_chunk, 20)
    assert r["first_chunk_us_per_it"] == 170
    assert abs(r["last_chunk_us_per_it"] - 147.0) < 1e-9
    assert r["seconds"] >= 0.05
    n = r["iterations"] // 20
    assert abs(per_it[n - 1] - per_it[n - 2]) <= 0.01 * per_it[n - 2]


def test_settle_respects_the_time_cap(monkeypatch):
    # never agreeing chunks end at max_s
    per_it = [100 + (i % 2) * 50 for i in range(1000)]
    now, run_chunk = _fake_chunks([x * 20e-3 for x in per_it])
    monkeypatch.setattr(bench.time, "perf_counter", now)
    r = bench.settle_clocks(run_chunk, 20, max_s=1.0)
    assert r["seconds"] >= 1.0 and r["seconds"] < 1.0 + 150 * 20e-3


def test_settle_fixed_chunks_is_exact(monkeypatch):
    # strips that exchange every iteration: the same count on every rank
    now, run_chunk = _fake_chunks([1e-3] * 20)
    monkeypatch.setattr(bench.time, "perf_counter", now)
    assert bench.settle_clocks(run_chunk, 20, fixed_chunks=8)["iterations"] == 160


def test_c2_algorithmic_work_model():
    # 292 L K^2 flops and (18 L + 2) S bytes per node and iteration
    assert bench.algorithmic_flops_per_node("mixture", 1, 9) == 292 * 81
    assert bench.algorithmic_bytes_per_node("mixture", 1, 8) == 160
