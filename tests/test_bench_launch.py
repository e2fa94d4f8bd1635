"""bench.py's multi-rank path on the CPU (no GPU): `--gpus 2` without a launcher starts two ranks
through torch.distributed.run (gloo), the ranks take contiguous shards of the global batch
(shard_range), and rank 0 reports sum-of-units / max-wall and the all-reduced check count --
the aggregation the 1/2/4/8-GPU PBS/s line uses (model
tfhe/benches/core_crypto/pbs_bench.rs:430-549)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=150):
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    if extra_env:
        env.update(extra_env)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_gpus_flag_launches_ranks_and_aggregates(world):
    p, lines = _run(["--gpus", str(world), "--launch-selftest", "--steps", "3", "--warmup", "1", "--batch", "10"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout          # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["world_size"] == world and d["backend"] == "gloo"
    G = 10 * world
    assert d["config"]["global_batch"] == G
    shards = d["config"]["shards"]
    assert shards[0][0] == 0 and shards[-1][1] == G
    assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))
    assert d["check"] == {"decrypted_ok": G, "of": G}
    assert d["units_total"] == G * 3
    # value = all units / the SLOWEST rank's wall (rank world-1 sleeps 0.02*world s per step)
    assert d["wall_max_s"] >= 3 * 0.02 * world
    assert abs(d["value"] - d["units_total"] / d["wall_max_s"]) < 1e-6 * d["value"]


def test_gpus_mismatch_with_world_is_an_error():
    p, _ = _run(["--gpus", "2", "--launch-selftest"], extra_env={"WORLD_SIZE": "1"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in (p.stderr + p.stdout)


@pytest.mark.timeout(180)
def test_other_workloads_failed_child_is_reported_not_fatal(monkeypatch):
    """The default run's side measurements (other_workloads): a child that cannot run (no GPU
    here) is reported as an error entry with its wall time; the caller keeps going."""
    import argparse
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setattr(bench, "OTHER_WORKLOADS", (("2_2ks", "2_2ks", {"steps": 1}),))
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")  # the child must fail fast on this CPU box
    res = bench.other_workloads(argparse.Namespace(seed=1))
    assert set(res) == {"2_2ks", "ctx_devices"}  # ctx_devices: the one-process multi-device entry, always run
    for k in res:
        assert "error" in res[k] and res[k]["wall_s"] > 0


@pytest.mark.timeout(240)
def test_multi_rank_default_run_merges_every_configuration():
    """The driver's N > 1 default run: every rank runs each other configuration in-process on the
    job's process group (keys broadcast, shards, barrier-bracketed timing, max wall over ranks)
    before the headline, and rank 0 prints ONE line whose other_workloads entries carry the world
    size they ran at (stub steps on gloo here; on the GPU box these are the PBS workloads)."""
    p, lines = _run(["--gpus", "2", "--launch-selftest", "--steps", "2", "--warmup", "1", "--batch", "8"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    names = [w[0] for w in bench.OTHER_WORKLOADS]
    assert {"mb3", "mul32", "4_4", "4_4_full"} <= set(names)
    ow = d["other_workloads"]
    assert list(ow) == names
    for name, params, opts in bench.OTHER_WORKLOADS:
        e = ow[name]
        assert e["world_size"] == 2 and e["n_gpus"] == 2, (name, e)
        assert e["steps"] == opts["steps"]
        if opts.get("global_batch"):   # config 3 at its stated size: a fixed total split over the ranks
            assert e["batch"] == opts["global_batch"] and e["scaling"] == "strong"
        else:
            assert e["batch"] == 16 and e["scaling"] == "weak"
        assert e["check"]["decrypted_ok"] == e["check"]["of"] == e["batch"]
    assert d["world_size"] == 2 and d["check"]["decrypted_ok"] == 16


@pytest.mark.timeout(240)
def test_multi_rank_workload_over_budget_still_prints_the_line():
    """N > 1: one configuration stalls (stub sleeping far past BENCH_WORKLOAD_BUDGET_S): every
    rank's watchdog fires, rank 0 prints the merged line -- the headline (measured first), the
    configurations measured before the stall, and that entry marked as an error -- and the job
    exits non-zero instead of hanging the multi-GPU run."""
    p, lines = _run(["--gpus", "2", "--launch-selftest", "--steps", "2", "--warmup", "1", "--batch", "8"],
                    extra_env={"BENCH_SELFTEST_STALL": "mb2", "BENCH_WORKLOAD_BUDGET_S": "4"})
    assert p.returncode != 0
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["check"]["decrypted_ok"] == 16            # the headline
    ow = d["other_workloads"]
    assert "error" in ow["mb2"] and "budget" in ow["mb2"]["error"]
    assert d["other_workloads_errors"] == ["mb2"]
    assert ow["mb3"]["world_size"] == 2 and "error" not in ow["mb3"]   # ran before the stall
    assert "4_4" not in ow                               # never started
