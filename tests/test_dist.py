"""Multi-rank path on CPU: shard planning, the socket control plane, and a world-size-2
``gloo`` run whose rank-ordered gather equals the reference's frame-ordered np.vstack
(LMC:887-889).  The per-rank compute here is the oracle (test-only); on GPUs it is the HIP
kernel and the gather is RCCL (tests/test_gpu_parity.py covers the single-rank RCCL path)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, pkg


def test_plan_shards_properties():
    d = pkg().dist
    rng = np.random.default_rng(0)
    for _ in range(50):
        F = int(rng.integers(0, 40))
        counts = rng.integers(0, 5000, F)
        for W in (1, 2, 3, 4, 8):
            b = d.plan_shards(counts, W)
            assert len(b) == W + 1 and b[0] == 0 and b[-1] == F
            assert np.all(np.diff(b) >= 0)
            if counts.sum() > 0 and F >= W:
                per = [counts[b[r]:b[r + 1]].sum() for r in range(W)]
                assert max(per) <= counts.sum() / W + counts.max() + 1
    assert d.plan_shards([100] * 8, 8).tolist() == list(range(9))
    with pytest.raises(ValueError):
        d.plan_shards([1], 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rdv_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import importlib
    d = importlib.import_module("livox-motion-compensation-sim_amd").dist
    r = d.Rendezvous(rank, world, "127.0.0.1", port, timeout=60)
    got = r.allgather({"rank": rank, "n": rank * 10})
    mx = r.max(float(rank) * 1.5)
    r.barrier()
    blob = r.broadcast_bytes(b"uid-" + bytes(range(124)) if rank == 0 else None)
    r.close()
    q.put((rank, got, mx, blob))


@pytest.mark.parametrize("world", [3, 8])
def test_rendezvous_processes(world):
    """The control plane at 3 ranks and at the 8 of one MI355X node (bench.py --gpus 8)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rdv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, mx, blob in res:
        assert got == [{"rank": r, "n": r * 10} for r in range(world)]
        assert mx == (world - 1) * 1.5
        assert blob == b"uid-" + bytes(range(124))


def _gloo_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import importlib
    import torch.distributed as dist
    from oracle import restatement as R
    from oracle import synth
    m = importlib.import_module("livox-motion-compensation-sim_amd")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sim = m.LiDARMotionSimulator({"duration": 12.0, "trajectory_type": "figure_eight", "max_speed": 12.0})
    tr = sim.add_sensor_noise(sim.generate_trajectory())
    times = sim.lidar_times()
    counts = np.array([(997 * (f + 3)) % 4000 for f in range(len(times))], np.int64)
    b = m.dist.plan_shards(counts, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    x, y, z, i, t = synth.synth_batch(counts[lo:hi], seed=5, frame_id_base=lo)
    pts = np.column_stack([x, y, z, i]).astype(np.float64)
    offs = np.concatenate([[0], np.cumsum(counts[lo:hi])])
    shard = [pts[offs[k]:offs[k + 1]] for k in range(hi - lo)]
    aligned = R.align_frames(shard, tr, times[lo:hi])
    local = R.merge_aligned(aligned) if aligned else np.zeros((0, 4))
    parts = [None] * world
    dist.all_gather_object(parts, local)
    dist.destroy_process_group()
    if rank == 0:
        x, y, z, i, t = synth.synth_batch(counts, seed=5, frame_id_base=0)
        allp = np.column_stack([x, y, z, i]).astype(np.float64)
        offs = np.concatenate([[0], np.cumsum(counts)])
        full = R.merge_aligned(R.align_frames([allp[offs[k]:offs[k + 1]] for k in range(len(counts))], tr, times))
        q.put(bool(np.array_equal(np.vstack(parts), full)))
    else:
        q.put(True)


def test_gloo_world2_shard_and_gather_equals_vstack():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res)


def _blocked(rows, counts, C):
    """Dense (N, C) rows of ragged frames -> the batch's blocked column layout."""
    counts = np.asarray(counts, np.int64)
    pad = (counts + 255) // 256 * 256
    poff = np.concatenate([[0], np.cumsum(pad)])
    doff = np.concatenate([[0], np.cumsum(counts)])
    flat = np.zeros(int(poff[-1]) * C, np.float32)
    for f in range(len(counts)):
        p = poff[f] + np.arange(counts[f])
        for c in range(C):
            flat[((p >> 8) * C + c) * 256 + (p & 255)] = rows[doff[f]:doff[f + 1], c]
    return flat, int(poff[-1])


def _unblocked(flat, counts, C):
    counts = np.asarray(counts, np.int64)
    pad = (counts + 255) // 256 * 256
    poff = np.concatenate([[0], np.cumsum(pad)])
    out = []
    for f in range(len(counts)):
        p = poff[f] + np.arange(counts[f])
        out.append(np.stack([flat[((p >> 8) * C + c) * 256 + (p & 255)] for c in range(C)], 1))
    return np.concatenate(out) if out else np.zeros((0, C), np.float32)


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
def test_gather_plan_of_sharded_run_equals_vstack(world):
    """The library's gather plan (mc_gather_plan, the host half of mc_comm_gather_batch) applied to
    plan_shards' point-balanced frame shards with numpy copies in place of the RCCL receives: the
    merged batch, read back in frame order, is np.vstack of the ranks' aligned clouds (LMC:887-889).
    Every root, 4- and 5-column shards (t_ns carried or not), empty shards, ragged frames."""
    d = pkg().dist
    rng = np.random.default_rng(world)
    for trial in range(6):
        F = int(rng.integers(0, 30))
        counts = rng.choice([0, 1, 7, 255, 256, 257, 3000, 10_001], F)
        b = d.plan_shards(counts, world)
        shard_counts = [counts[b[r]:b[r + 1]] for r in range(world)]
        merged_C = int(rng.choice([4, 5]))
        Cs = [5 if merged_C == 5 else int(rng.choice([4, 5])) for _ in range(world)]
        rows = [rng.standard_normal((int(sc.sum()), 5)).astype(np.float32) for sc in shard_counts]
        shards, P = [], []
        for r in range(world):
            flat, pr = _blocked(rows[r], shard_counts[r], Cs[r])
            shards.append(flat)
            P.append(pr)
        root = int(rng.integers(0, world))
        plan = d.gather_plan(P, Cs, sum(P), merged_C, root=root)
        merged = np.full(sum(P) * merged_C, np.nan, np.float32)
        stage = np.full(plan["stage_values"], np.nan, np.float32)
        for q in range(world):          # the receives
            if q == root or P[q] == 0:
                continue
            n = Cs[q] * P[q]
            if plan["stage_offset"][q] >= 0:
                stage[plan["stage_offset"][q]:plan["stage_offset"][q] + n] = shards[q]
            else:
                merged[plan["offset"][q] * merged_C:plan["offset"][q] * merged_C + n] = shards[q]
        for q in range(world):          # the root's own shard and the re-pitches
            if P[q] == 0 or (q != root and plan["stage_offset"][q] < 0):
                continue
            src = shards[q] if q == root else stage[plan["stage_offset"][q]:plan["stage_offset"][q] + Cs[q] * P[q]]
            blocks = src.reshape(P[q] // 256, Cs[q], 256)[:, :merged_C]
            o = plan["offset"][q] * merged_C
            merged[o:o + P[q] * merged_C] = blocks.reshape(-1)
        got = _unblocked(merged, counts, merged_C)
        want = np.vstack([rw[:, :merged_C] for rw in rows]) if rows else np.zeros((0, merged_C))
        assert np.array_equal(got, want), (world, trial, root, Cs, merged_C)


def test_gather_plan_rejects_narrow_shards_and_bad_totals():
    d = pkg().dist
    with pytest.raises(ValueError, match="columns"):
        d.gather_plan([256, 512], [4, 5], 768, 5)          # t_ns would be left undefined
    with pytest.raises(ValueError, match="padded points"):
        d.gather_plan([256, 512], [5, 5], 1024, 4)
    with pytest.raises(ValueError, match="block"):
        d.gather_plan([100], [4], 100, 4)
    with pytest.raises(ValueError, match="root"):
        d.gather_plan([256], [4], 256, 4, root=1)
    assert d.gather_plan([0, 256], [4, 4], 256, 4)["offset"].tolist() == [0, 0]


# ---------------------------------------------------------------------------------------------
# bench.py --gpus N without torchrun: the bench launches its own rank processes
# ---------------------------------------------------------------------------------------------
def _bench(args, env_extra=None, timeout=120):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launch_control_plane(n):
    """python bench.py --gpus N (no torchrun env): N rank processes rendezvous over the control
    plane, rank 0 prints one line (the driver's 8-GPU command form must not run 1 rank)."""
    rc, line, err = _bench(["--gpus", str(n), "--control-plane-only"])
    assert rc == 0, err
    assert line["world"] == n and line["launched_by"] == "bench.py"
    assert [r["rank"] for r in line["ranks"]] == list(range(n))
    assert [r["local_rank"] for r in line["ranks"]] == list(range(n))
    assert len({r["pid"] for r in line["ranks"]}) == n
    assert line["max_over_ranks"] == n - 1


def test_bench_self_launch_fails_when_a_rank_fails():
    rc, line, _ = _bench(["--gpus", "3", "--control-plane-only"],
                         {"MCBENCH_FAIL_RANK": "2", "MCBENCH_RDV_TIMEOUT": "5"})
    assert rc != 0 and line is None


def test_bench_self_launch_timeout_kills_every_rank():
    rc, line, err = _bench(["--gpus", "2", "--control-plane-only", "--launch-timeout", "4"],
                           {"MCBENCH_HANG_RANK": "1"})
    assert rc == 124 and line is None and "timeout" in err
