"""Multi-GPU sharding of the frame batch and the merged-cloud gather.

Frames are independent (LMC:802-832 carries no state across frames), so a run shards as
contiguous, point-balanced frame ranges — one process per GPU, no collective on the data path.
The one exchange step is the reference's merge (np.vstack, LMC:887-889): concatenating the
ranks' shards in rank order reproduces it, done as one ragged RCCL gather over xGMI
(``mc_comm_gather_batch``).

Control plane (rank/world from torchrun's env; barrier, max-over-ranks, RCCL unique-id
broadcast) is a small TCP star on MASTER_ADDR:MASTER_PORT+1 or the next free port (stdlib sockets — the GPU
processes load no torch).  ``Rendezvous`` works on CPU, which the world-size-2 tests use.
"""
from __future__ import annotations

import ctypes
import json
import os
import socket
import struct
import sys
import time
from ctypes import c_char, c_double, c_void_p

import numpy as np

from . import _lib
from ._lib import check, ptr


def plan_shards(counts, world_size: int) -> np.ndarray:
    """Contiguous frame ranges balanced by point count: rank r owns frames [b[r], b[r+1]).

    b[r] = first frame whose preceding-points prefix reaches r * total / world_size, so the
    rank-ordered concatenation of the shards is the frame-ordered merge.
    """
    counts = np.asarray(counts, dtype=np.int64)
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    prefix = np.concatenate([[0], np.cumsum(counts)])
    total = prefix[-1]
    F = len(counts)
    bounds = [0]
    for r in range(1, world_size):
        target = (total * r) // world_size
        b = int(np.searchsorted(prefix, target, side="left"))
        if total == 0:
            b = (F * r) // world_size
        bounds.append(min(max(b, bounds[-1]), F))
    bounds.append(F)
    return np.asarray(bounds, dtype=np.int64)


def env_rank() -> tuple:
    """(rank, local_rank, world_size) from the torchrun environment (defaults 0, 0, 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


# ---------------------------------------------------------------------------------------------
# control plane
# ---------------------------------------------------------------------------------------------
def _send(sock, payload: bytes):
    sock.sendall(struct.pack("!Q", len(payload)) + payload)


def _recv(sock) -> bytes:
    head = b""
    while len(head) < 8:
        chunk = sock.recv(8 - len(head))
        if not chunk:
            raise ConnectionError("peer closed")
        head += chunk
    n = struct.unpack("!Q", head)[0]
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


def _recv_exact(sock, n: int) -> bytes:
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return buf


_MAGIC = b"MCRDV\x00\x00\x01"   # rank 0's greeting, sent first on every accepted connection
_PORT_TRIES = 32                    # rank 0 takes the first free port of base .. base + 31
_GREETING_WAIT = 5.0                # seconds a rank waits for the greeting before trying the next port


class Rendezvous:
    """Star-topology control channel: rank 0 accepts world_size-1 connections.

    Rank 0 listens on MASTER_PORT + 1 (or ``port``), or on the next free port of the 32 above it
    when that one is taken (say by a service of the launcher); it greets each connection with a
    magic word before anything else, and a rank sends its (world size, rank) only after that
    greeting, so a rank that reached a foreign listener (no greeting within ``_GREETING_WAIT``)
    closes it and tries the next port, and a connection the rank gave up on before rank 0 accepted
    it never registers (its rank word never arrives)."""

    def __init__(self, rank: int, world_size: int, addr: str | None = None, port: int | None = None,
                 timeout: float = 300.0):
        self.rank, self.world_size = rank, world_size
        self.peers = {}
        self.sock = None
        if world_size == 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        base = port if port is not None else int(os.environ.get("MASTER_PORT", "29500")) + 1
        ports = [base + k for k in range(_PORT_TRIES) if base + k < 65536]
        deadline = time.time() + timeout
        if rank == 0:
            srv, err = None, None
            for p in ports:
                srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                try:
                    srv.bind((addr, p))
                    break
                except OSError as e:
                    srv.close()
                    srv, err = None, e
            if srv is None:
                raise OSError(f"rendezvous: no free port in {ports[0]}..{ports[-1]}: {err}")
            self.port = srv.getsockname()[1]
            srv.listen(max(world_size, 16))
            try:
                while len(self.peers) < world_size - 1:
                    left = deadline - time.time()
                    if left <= 0:
                        raise TimeoutError(f"rendezvous: {len(self.peers) + 1} of {world_size} ranks arrived")
                    srv.settimeout(left)
                    conn, _ = srv.accept()
                    try:
                        conn.settimeout(10.0)
                        conn.sendall(_MAGIC)
                        ws, r = struct.unpack("!II", _recv_exact(conn, 8))
                        ok = ws == world_size and 0 < r < world_size and r not in self.peers
                    except (OSError, struct.error):
                        ok = False
                    if not ok:
                        conn.close()
                        continue
                    conn.settimeout(timeout)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    self.peers[r] = conn
            finally:
                srv.close()
        else:
            k = 0
            while True:
                p = ports[k % len(ports)]
                k += 1
                s = None
                try:
                    s = socket.create_connection((addr, p), timeout=1.0)
                    s.settimeout(_GREETING_WAIT)
                    if _recv_exact(s, len(_MAGIC)) == _MAGIC:
                        s.sendall(struct.pack("!II", world_size, rank))
                        break
                except OSError:
                    pass
                if s is not None:
                    s.close()
                if time.time() > deadline:
                    raise TimeoutError(f"rendezvous: rank {rank} found no rank 0 on {ports[0]}..{ports[-1]}")
                if k % len(ports) == 0:
                    time.sleep(0.05)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.sock = s
            self.port = p

    def allgather(self, obj):
        """Every rank gets the rank-ordered list of every rank's JSON-serialisable obj."""
        if self.world_size == 1:
            return [obj]
        if self.rank == 0:
            vals = [obj] + [None] * (self.world_size - 1)
            for r, c in self.peers.items():
                vals[r] = json.loads(_recv(c))
            blob = json.dumps(vals).encode()
            for c in self.peers.values():
                _send(c, blob)
            return vals
        _send(self.sock, json.dumps(obj).encode())
        return json.loads(_recv(self.sock))

    def broadcast_bytes(self, data: bytes | None) -> bytes:
        if self.world_size == 1:
            return data
        if self.rank == 0:
            for c in self.peers.values():
                _send(c, data)
            return data
        return _recv(self.sock)

    def barrier(self):
        self.allgather(0)

    def max(self, value: float) -> float:
        return max(self.allgather(float(value)))

    def close(self):
        for c in self.peers.values():
            c.close()
        if self.sock is not None:
            self.sock.close()
        self.peers = {}
        self.sock = None


# ---------------------------------------------------------------------------------------------
# RCCL data plane
# ---------------------------------------------------------------------------------------------
class RcclComm:
    """RCCL communicator over the ranks of ``rdv`` (unique id broadcast through it)."""

    def __init__(self, ctx, rdv: Rendezvous):
        self.lib = ctx.lib
        self.ctx = ctx
        self.rank, self.world_size = rdv.rank, rdv.world_size
        uid = (c_char * 128)()
        if rdv.rank == 0:
            check(self.lib.mc_comm_unique_id(uid), "comm_unique_id")
        data = rdv.broadcast_bytes(bytes(uid) if rdv.rank == 0 else None)
        uid = (c_char * 128).from_buffer_copy(data)
        h = c_void_p()
        # librccl prints its version banner on stdout during init; keep stdout for the caller's
        # output (bench.py's one JSON line) by pointing fd 1 at stderr meanwhile
        sys.stdout.flush()
        saved = os.dup(1)
        try:
            os.dup2(2, 1)
            rc = self.lib.mc_comm_init(ctx.handle, rdv.world_size, rdv.rank, uid, ctypes.byref(h))
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        check(rc, "comm_init")
        self.handle = h

    def gather_batch(self, local, merged=None, root: int = 0):
        """Ragged gather of every rank's batch columns into ``merged`` on ``root`` (rank order)."""
        check(self.lib.mc_comm_gather_batch(self.handle, local.handle, root,
                                            merged.handle if merged is not None else None), "gather_batch")
        return merged

    def allreduce_max(self, values) -> np.ndarray:
        v = np.ascontiguousarray(np.atleast_1d(values), dtype=np.float64).copy()
        check(self.lib.mc_comm_allreduce_max_f64(self.handle, ptr(v, c_double), len(v)), "allreduce_max")
        return v

    def close(self):
        if self.handle:
            self.lib.mc_comm_destroy(self.handle)
            self.handle = None


def gather_plan(padded, columns, merged_padded: int, merged_columns: int, root: int = 0) -> dict:
    """The plan ``mc_comm_gather_batch`` follows (host only, csrc/plan.cpp): per rank the shard's
    first padded point in the merged batch (rank order == np.vstack order, LMC:887-889) and its
    value offset in the root's staging area (-1: received in place); raises ValueError for an
    invalid plan (sizes that do not add up, a shard narrower than the merged batch)."""
    lib = _lib.load()
    P = np.ascontiguousarray(padded, dtype=np.int64)
    C = np.ascontiguousarray(columns, dtype=np.int64)
    if P.shape != C.shape or P.ndim != 1:
        raise ValueError("padded / columns: one entry per rank")
    off = np.zeros(len(P), np.int64)
    soff = np.zeros(len(P), np.int64)
    sv = np.zeros(1, np.int64)
    check(lib.mc_gather_plan(len(P), int(root), ptr(P, ctypes.c_int64), ptr(C, ctypes.c_int64), int(merged_padded),
                             int(merged_columns), ptr(off, ctypes.c_int64), ptr(soff, ctypes.c_int64),
                             ptr(sv, ctypes.c_int64)), "gather_plan")
    return {"offset": off, "stage_offset": soff, "stage_values": int(sv[0])}


def gather_batches(ctx, shards, root: int = 0, merged=None):
    """One process, several shard batches of ``ctx`` merged as ``gather_merged`` merges ranks'
    shards (same plan, staging and re-pitch; device copies in place of the RCCL receives).
    ``merged`` defaults to a 4-column batch of the concatenated frame counts."""
    if merged is None:
        merged = ctx.batch(np.concatenate([np.asarray(b.counts, np.int64) for b in shards]))
    arr = (c_void_p * len(shards))(*[b.handle.value for b in shards])
    check(ctx.lib.mc_gather_batches(ctx.handle, len(shards), arr, int(root), merged.handle), "gather_batches")
    return merged


def gather_merged(ctx, comm: RcclComm, rdv: Rendezvous, local, root: int = 0):
    """Merged aligned cloud of all ranks on ``root`` (None elsewhere) — the LMC:888 vstack."""
    all_counts = rdv.allgather([int(c) for c in local.counts])
    merged = None
    if rdv.rank == root:
        merged = ctx.batch(np.concatenate([np.asarray(c, np.int64) for c in all_counts]))
    comm.gather_batch(local, merged, root)
    return merged
