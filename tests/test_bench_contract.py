"""CPU: the bench line's honesty guards.

* roofline.traffic (PMC HBM bytes) is attached only when the traffic file was
  measured on the same kernel instantiation of the same libpipck.so build
  (a substring match let another template's traffic ride along);
* an N-rank run cannot claim more GPUs than it ran on (--share-gpus or refuse);
* the packed-batch bounds check cannot go stale when the allocator reuses an
  address.
"""
import pytest

import bench
from pip_amd import engine, shard

K = ("void pipck::k_packed<false, 32, true, true>(unsigned char const*, unsigned short const*, unsigned long const*, "
     "unsigned long, unsigned int const*, unsigned int, unsigned int const*, unsigned long, unsigned short*, "
     "unsigned char*, unsigned int)")
SHA = "ab" * 32


def record(**kw):
    t = {"kernel": K, "lib_sha256": SHA, "algorithmic_bytes_per_launch": 8291632672, "arena_stride": 0,
         "hbm_bytes_per_launch": 8458390912}
    t.update(kw)
    return t


def test_traffic_attached_on_exact_match():
    got, why = bench.match_traffic(record(), K, SHA, 8291632672, 0)
    assert got == 8458390912 and why == "match"


@pytest.mark.parametrize("field,value", [
    # another instantiation of the same template (ring 24 instead of 32): the r02 hole
    ("kernel", K.replace("<false, 32, true, true>", "<false, 24, true, true>")),
    ("kernel", K.replace("<false, 32, true, true>", "<false, 32, true, false>")),
    ("kernel", "void pipck::k_packed"),  # a prefix is not the kernel
    ("lib_sha256", "cd" * 32),             # same name, another build
    ("lib_sha256", None),                  # a pre-r03 file without a build hash
    ("algorithmic_bytes_per_launch", 8291632672 + 16),
    ("arena_stride", 20),
])
def test_mismatched_traffic_yields_null(field, value):
    got, why = bench.match_traffic(record(**{field: value}), K, SHA, 8291632672, 0)
    assert got is None
    assert field in why


def test_committed_traffic_files_carry_kernel_and_build():
    """Every committed traffic file names its full kernel instantiation, so the
    bench can bind it exactly; files predating the build hash are simply never
    attached (match_traffic above)."""
    import json
    from pathlib import Path

    files = sorted((Path(bench.ROOT) / "profiles").glob("traffic_cfg*.json"))
    assert files
    for f in files:
        t = json.loads(f.read_text())
        assert t["kernel"].startswith("void pipck::k_") and "(" in t["kernel"], f.name


@pytest.mark.parametrize("world,n_dev,share,ok", [  # world = ranks on the node
    (1, 1, False, True), (8, 8, False, True), (4, 8, False, True),
    (2, 1, False, False), (8, 1, False, False), (8, 4, False, False),
    (4, 1, True, True), (8, 4, True, True), (1, 0, False, False), (1, 0, True, False),
])
def test_ranks_never_exceed_visible_gpus_without_share(world, n_dev, share, ok):
    if ok:
        devs = [shard.device_for_rank(r, world, n_dev, share) for r in range(world)]
        assert all(0 <= d < n_dev for d in devs)
        if world <= n_dev:
            assert len(set(devs)) == world  # one GPU per rank
    else:
        with pytest.raises(ValueError):
            shard.device_for_rank(world - 1, world, n_dev, share)


def test_bench_refuses_more_ranks_than_gpus_before_timing(monkeypatch, capsys):
    """Under torch.distributed.run with WORLD_SIZE=2 on a machine with no (or one)
    GPU and no --share-gpus, the rank exits non-zero before any timed work."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    rc = bench.main(["--gpus", "1", "--steps", "1", "--warmup", "0"])
    assert rc == 3
    assert "no visible GPU" in capsys.readouterr().err


class TestPackedBoundsCache:
    """engine._check_packed caches the index total on the index tensor object and
    its version, so neither an in-place rewrite nor a reused address skips the check."""

    def test_in_place_rewrite_is_rechecked(self):
        torch = pytest.importorskip("torch")
        lens = torch.zeros(100, dtype=torch.int16)
        tc = torch.tensor([0, 10, 20], dtype=torch.int64)
        arena = torch.empty(320, dtype=torch.uint8)
        engine._check_packed(arena, lens, tc, 100)
        tc[2] = 30  # same object, same address: a larger total
        with pytest.raises(ValueError):
            engine._check_packed(arena, lens, tc, 100)

    def test_new_index_at_a_reused_address_is_rechecked(self):
        torch = pytest.importorskip("torch")
        lens = torch.zeros(100, dtype=torch.int16)
        arena = torch.empty(320, dtype=torch.uint8)
        for total in (10, 20, 40):  # freed and reallocated each time (often at the same address)
            tc = torch.tensor([0, total // 2, total], dtype=torch.int64)
            if 16 * total <= 320:
                engine._check_packed(arena, lens, tc, 100)
            else:
                with pytest.raises(ValueError):
                    engine._check_packed(arena, lens, tc, 100)
            del tc

    def test_smaller_arena_is_rechecked(self):
        torch = pytest.importorskip("torch")
        lens = torch.zeros(100, dtype=torch.int16)
        tc = torch.tensor([0, 10, 20], dtype=torch.int64)
        engine._check_packed(torch.empty(320, dtype=torch.uint8), lens, tc, 100)
        with pytest.raises(ValueError):
            engine._check_packed(torch.empty(319, dtype=torch.uint8), lens, tc, 100)


def test_aggregate_is_span_from_earliest_start_to_latest_end():
    """Σ units / (max end - min start); a late starter lengthens
    the span even when every rank's own elapsed time is the same."""
    ms = 1_000_000
    even = shard.aggregate([0, 0], [50 * ms, 50 * ms], [1e9, 1e9], 10)
    assert even["span_s"] == even["max_rank_s"] == 0.05 and even["rate"] == even["rate_max_rank"] == 4e11
    skewed = shard.aggregate([0, 100 * ms], [50 * ms, 150 * ms], [1e9, 1e9], 10)
    assert skewed["max_rank_s"] == 0.05 and skewed["span_s"] == 0.15
    assert skewed["start_skew_ms"] == 100 and skewed["end_skew_ms"] == 100
    assert skewed["rate"] == pytest.approx(2e10 / 0.15) and skewed["rate_max_rank"] == 4e11


_SKEW_SCRIPT = """
import json, sys, time
sys.path.insert(0, {root!r})
from pip_amd import shard
env = shard.dist_env()
shard.init_control_plane(env)
steps, step_s, skew_s = 5, 0.02, {skew}
t0, t1 = shard.timed_steps(env, steps, lambda i: time.sleep(step_s), lambda: None,
                           before_start=lambda: time.sleep(env.rank * skew_s))
clocks = shard.gather_ints(env, [t0, t1])
agg = shard.aggregate([c[0] for c in clocks], [c[1] for c in clocks], [1e9] * env.world, steps)
if env.rank == 0:
    print("AGG " + json.dumps(agg), flush=True)
shard.shutdown(env)
"""


@pytest.mark.parametrize("world", [2, 4])
def test_injected_start_skew_lowers_the_aggregate(tmp_path, capfd, world):
    """gloo ranks on one host whose timed starts are skewed after the barrier
    (rank r waits r x 200 ms, as bench.py --start-skew-ms does): the reported
    aggregate drops by the skew, while the max-over-ranks elapsed time would
    not see it.  Unskewed, the two agree within the scheduling noise of
    several processes on a busy CPU (a 50-ms bound failed once under pytest -n 4)."""
    import json
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parents[1])
    got = {}
    for skew in (0.0, 0.2):
        script = tmp_path / f"skew{skew}.py"
        script.write_text(_SKEW_SCRIPT.format(root=root, skew=skew))
        assert shard.spawn_ranks(world, [sys.executable, str(script)]) == 0
        out = capfd.readouterr().out
        got[skew] = json.loads(next(ln for ln in out.splitlines() if ln.startswith("AGG "))[4:])
    flat, skewed = got[0.0], got[0.2]
    want_skew = (world - 1) * 200
    assert flat["start_skew_ms"] < 150 and flat["span_s"] < flat["max_rank_s"] + 0.15
    assert want_skew - 50 < skewed["start_skew_ms"] < want_skew + 150
    # the span covers the skew and a whole rank's run (the slowest rank need
    # not be the late starter on a busy CPU, so not max_rank_s + skew)
    assert skewed["span_s"] >= skewed["start_skew_ms"] / 1e3 + 0.1 - 0.005
    assert skewed["span_s"] > skewed["max_rank_s"] + 0.1
    assert skewed["rate"] < 0.75 * skewed["rate_max_rank"]
    assert skewed["rate"] == pytest.approx(world * 1e9 * 5 / skewed["span_s"])


def test_cpu_sample_falls_back_to_the_memory_the_host_has(monkeypatch):
    """the CPU baseline's BASELINE.md sample (up to ~9 GB) is cut to
    what half of MemAvailable holds, never below 4K packets; the full plan when it
    fits or when /proc/meminfo cannot be read."""
    from pip_amd.workloads import BY_CFG

    w = BY_CFG[5]
    per = bench.host_bytes_per_packet(w)
    assert per >= w.stride
    monkeypatch.setattr(bench, "mem_available", lambda: 64 << 30)
    assert bench.sample_that_fits(1 << 20, per) == 1 << 20
    monkeypatch.setattr(bench, "mem_available", lambda: 4 << 30)
    n = bench.sample_that_fits(1 << 20, per)
    assert 4096 <= n < 1 << 20 and n * per <= 2 << 30
    monkeypatch.setattr(bench, "mem_available", lambda: 0)
    assert bench.sample_that_fits(1 << 20, per) == 1 << 20
