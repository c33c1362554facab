"""Multi-rank path on CPU: shard planning, the socket control plane, and ``gloo`` runs of the
merged-cloud gather (LMC:887-889 np.vstack).  Each rank holds its frame shard in the product's
blocked-CSR batch layout; the root assembles the merged batch at the offsets of the library's own
gather plan (mc_gather_plan, the host half of mc_comm_gather_batch) from point-to-point
sends / receives — the transfers mc_comm_gather_batch issues as ncclSend / ncclRecv — including
shards whose column count differs (t_ns carried) and is re-pitched.  On GPUs the same plan drives
RCCL (tests/test_gpu_gather_issue.py covers the device copies / re-pitch in one process), and the
library's own C++ gather sequence (csrc/gather.cpp) runs between forked processes over a socket
transport (worlds 2, 3, 8)."""
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


@pytest.mark.parametrize("foreign", ["silent", "talks"])
def test_rendezvous_when_its_port_is_taken(foreign):
    """MASTER_PORT + 1 held by another service (a listener that never speaks, or one that answers
    with other bytes): rank 0 takes the next free port, the other ranks find it by its greeting."""
    import threading
    port = _free_port()
    other = socket.socket()
    other.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    other.bind(("127.0.0.1", port))
    other.listen(16)
    stop = threading.Event()

    def talker():
        other.settimeout(0.2)
        while not stop.is_set():
            try:
                c, _ = other.accept()
            except OSError:
                continue
            c.sendall(b"HTTP/1.1 400 Bad Request\r\n\r\n")
            c.close()
    t = threading.Thread(target=talker, daemon=True) if foreign == "talks" else None
    if t:
        t.start()
    try:
        world = 3
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
            assert blob == b"uid-" + bytes(range(124))
    finally:
        stop.set()
        if t:
            t.join()
        other.close()


def test_rendezvous_rank0_ignores_a_stray_connection():
    """A connection that answers rank 0's greeting with a wrong world size (or closes) is dropped;
    the real rank still registers."""
    import struct
    import threading
    d = pkg().dist
    port = _free_port()
    out = {}

    def root():
        r = d.Rendezvous(0, 2, "127.0.0.1", port, timeout=60)
        out["all"] = r.allgather("root")
        r.close()
    t = threading.Thread(target=root)
    t.start()
    for _ in range(200):   # the stray client: waits for the greeting, then lies about the world
        try:
            s = socket.create_connection(("127.0.0.1", port), timeout=1.0)
            break
        except OSError:
            import time
            time.sleep(0.02)
    assert s.recv(8) == d._MAGIC
    s.sendall(struct.pack("!II", 5, 1))
    s.close()
    s2 = socket.create_connection(("127.0.0.1", port), timeout=5.0)
    s2.close()                               # connects and leaves before sending its rank
    r1 = d.Rendezvous(1, 2, "127.0.0.1", port, timeout=60)
    got = r1.allgather("one")
    r1.close()
    t.join(timeout=60)
    assert got == ["root", "one"] and out["all"] == ["root", "one"]


def _gloo_worker(rank, world, root, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import importlib
    import torch
    import torch.distributed as dist
    from oracle import synth
    m = importlib.import_module("livox-motion-compensation-sim_amd")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sim = m.LiDARMotionSimulator({"duration": 12.0, "trajectory_type": "figure_eight", "max_speed": 12.0})
    F = len(sim.lidar_times())
    counts = np.array([(997 * (f + 3)) % 4000 for f in range(F)], np.int64)
    counts[3] = 0                                     # an empty frame inside a shard
    b = m.dist.plan_shards(counts, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    # this rank's frames: x, y, z, intensity (+ t_ns on odd ranks: a 5-column batch, re-pitched)
    x, y, z, i, t = synth.synth_batch(counts[lo:hi], seed=5, frame_id_base=lo)
    C = 5 if rank % 2 else 4
    rows = np.column_stack([x, y, z, i, t.astype(np.float32)])[:, :C]
    flat, P = _blocked(rows, counts[lo:hi], C)
    # shard sizes to every rank (a gather of two int64 per rank, as mc_comm_gather_batch's all-gather)
    meta = torch.tensor([P, C], dtype=torch.int64)
    metas = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(metas, meta)
    Ps = [int(v[0]) for v in metas]
    Cs = [int(v[1]) for v in metas]
    ok = True
    if rank == root:
        plan = m.dist.gather_plan(Ps, Cs, sum(Ps), 4, root=root)
        merged = np.full(sum(Ps) * 4, np.nan, np.float32)
        stage = np.full(max(plan["stage_values"], 1), np.nan, np.float32)
        for src in range(world):
            if src == root or Ps[src] == 0:
                continue
            n = Cs[src] * Ps[src]
            so = plan["stage_offset"][src]
            dst = stage[so:so + n] if so >= 0 else merged[plan["offset"][src] * 4:plan["offset"][src] * 4 + n]
            dist.recv(torch.from_numpy(dst), src=src)       # into the plan's place
        for r in range(world):                              # the root's own shard and the re-pitches
            if Ps[r] == 0 or (r != root and plan["stage_offset"][r] < 0):
                continue
            so = plan["stage_offset"][r]
            src_vals = flat if r == root else stage[so:so + Cs[r] * Ps[r]]
            o = plan["offset"][r] * 4
            merged[o:o + Ps[r] * 4] = src_vals.reshape(Ps[r] // 256, Cs[r], 256)[:, :4].reshape(-1)
        got = _unblocked(merged, counts, 4)
        x, y, z, i, t = synth.synth_batch(counts, seed=5, frame_id_base=0)
        frames = np.column_stack([x, y, z, i])
        offs = np.concatenate([[0], np.cumsum(counts)])
        want = np.vstack([frames[offs[f]:offs[f + 1]] for f in range(F)])   # LMC:888, frame order
        ok = bool(np.array_equal(got, want)) and not np.isnan(merged[:1]).any()
        ok = ok and any(plan["stage_offset"][r] >= 0 for r in range(world) if Cs[r] != 4 and r != root)
    elif P > 0:
        dist.send(torch.from_numpy(flat), dst=root)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("world,root", [(2, 0), (3, 2), (4, 1)])
def test_gloo_gather_of_blocked_shards_equals_vstack(world, root):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, root, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res


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
# the product's gather sequence (csrc/gather.cpp, behind mc_comm_gather_batch) between processes
# ---------------------------------------------------------------------------------------------
CSRC = os.path.join(ROOT, "livox-motion-compensation-sim_amd", "csrc")
SAN = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
       "-fno-omit-frame-pointer"]


@pytest.fixture(scope="module")
def gather_exe(tmp_path_factory):
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path_factory.mktemp("gs") / "gather_sockets"
    subprocess.run(["g++", *SAN, f"-I{CSRC}", os.path.join(ROOT, "tests", "host", "gather_sockets.cpp"),
                    os.path.join(CSRC, "gather.cpp"), os.path.join(CSRC, "plan.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    return str(exe)


def _run_sockets(exe, d, world, root, shard_counts, Cs, merged_counts, merged_C, shards):
    import subprocess
    P = [int(((np.asarray(sc, np.int64) + 255) // 256 * 256).sum()) for sc in shard_counts]
    mP = int(((np.asarray(merged_counts, np.int64) + 255) // 256 * 256).sum())
    lines = [f"{world} {root}", " ".join(map(str, [mP, merged_C, len(merged_counts), *merged_counts]))]
    for q in range(world):
        lines.append(" ".join(map(str, [P[q], Cs[q], len(shard_counts[q]), *shard_counts[q]])))
        shards[q].astype(np.float32).tofile(os.path.join(d, f"shard_{q}.bin"))
    with open(os.path.join(d, "meta.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, d], capture_output=True, text=True, timeout=120, env=env)
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    merged = None
    if r.returncode == 0:
        merged = np.fromfile(os.path.join(d, "merged.bin"), np.float32)
        assert merged.size == mP * merged_C
    return r, merged


@pytest.mark.parametrize("world,root", [(2, 0), (3, 1), (8, 5)])
def test_socket_transport_runs_the_product_gather_sequence(gather_exe, tmp_path, world, root):
    """mc_comm_gather_batch's own C++ sequence (plan all-gather, frame-hash check, grouped
    send / receive, the finishing copies and re-pitch: mcgather::run) between ``world`` forked
    processes over Unix sockets, under ASan + UBSan; the root's merged batch, read back in frame
    order, is np.vstack of the shards (LMC:887-889).  Shards come from plan_shards; one of them has
    5 columns (t_ns carried, re-pitched), one is empty, frames are ragged."""
    d = pkg().dist
    rng = np.random.default_rng(100 + world)
    counts = rng.choice([1, 7, 255, 256, 257, 3000, 10_001], 3 * world).astype(np.int64)
    b = d.plan_shards(counts, world)
    shard_counts = [counts[b[r]:b[r + 1]].tolist() for r in range(world)]
    empty = (root + 1) % world                      # an empty shard: its frames move to a neighbour
    nb = (empty + 1) % world
    if empty < nb:
        shard_counts[nb] = shard_counts[empty] + shard_counts[nb]
    else:
        shard_counts[nb] = shard_counts[nb] + shard_counts[empty]
    shard_counts[empty] = []
    order = sorted(range(world))
    merged_counts = [c for q in order for c in shard_counts[q]]
    Cs = [4] * world
    Cs[(root + 2) % world if world > 2 else nb] = 5       # a re-pitched 5-column shard
    rows = [rng.standard_normal((int(sum(sc)), 5)).astype(np.float32) for sc in shard_counts]
    shards = [_blocked(rows[q], shard_counts[q], Cs[q])[0] for q in range(world)]
    r, merged = _run_sockets(gather_exe, str(tmp_path), world, root, shard_counts, Cs, merged_counts, 4, shards)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert r.stdout.count("status 0") == world
    got = _unblocked(merged, merged_counts, 4)
    want = np.vstack([rw[:, :4] for rw in rows])
    assert np.array_equal(got, want)


def test_socket_transport_rejects_a_reordered_merge_on_every_rank(gather_exe, tmp_path):
    """Equal padded totals but the merged batch's frames in another order: every rank sees the same
    all-gathered plan words, rejects it (frame-hash check) and moves no data."""
    world, root = 3, 0
    shard_counts = [[300, 100], [512], [1]]
    merged_counts = [100, 300, 512, 1]
    Cs = [4, 4, 4]
    shards = [_blocked(np.ones((sum(sc), 4), np.float32), sc, 4)[0] for sc in shard_counts]
    r, merged = _run_sockets(gather_exe, str(tmp_path), world, root, shard_counts, Cs, merged_counts, 4, shards)
    assert r.returncode == 3, r.stdout
    assert r.stdout.count("status -1") == world and merged is None


def test_socket_transport_root_without_merged_batch_fails_everywhere(gather_exe, tmp_path):
    """A root that passes no merged batch still takes part in the plan all-gather, so every rank
    returns the error instead of waiting on the root forever."""
    import subprocess
    d = str(tmp_path)
    shard_counts = [[300], [256], [10]]
    shards = [_blocked(np.ones((sum(sc), 4), np.float32), sc, 4)[0] for sc in shard_counts]
    for q, sh in enumerate(shards):
        sh.tofile(os.path.join(d, f"shard_{q}.bin"))
    P = [512, 256, 256]
    lines = ["3 1", "-1 4 0"] + [" ".join(map(str, [P[q], 4, 1, shard_counts[q][0]])) for q in range(3)]
    with open(os.path.join(d, "meta.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    r = subprocess.run([gather_exe, d], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 3, r.stdout + r.stderr[-2000:]
    assert r.stdout.count("status -1 root needs a merged batch") == 3


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
