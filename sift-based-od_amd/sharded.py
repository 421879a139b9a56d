"""Database sharding across ranks (one process per GPU) -- SURVEY.md §8(e).

Rank r holds descriptor rows [lo_r, hi_r) of the database (the keypoint table and the
per-image table are replicated: they are ~8 % of the descriptor bytes and every rank
needs them to verify bins).  One query image is processed by every rank:

1. match the Nq queries against the local shard -> per query (d1^2, global idx1, d2^2)
2. ALL-GATHER those 12 B/query candidates; every rank merges them (lexicographic on
   (d^2, trainIdx), second = min of the rest) -- the ratio test is applied only AFTER
   this global merge (a per-shard ratio test would keep different matches)
3. each rank votes only for good matches whose trainIdx lies in its shard -> partial
   bin counts + first-touch ordinals; ALL-REDUCE (sum, min) gives the global histogram
   bit-exactly in any order
4. valid bins, members, PoseBin means and the affine verification then run identically
   on every rank (all inputs are replicated after 2 and 3).

Two communicators carry the two exchanges:

* :class:`RcclComm` -- RCCL over xGMI inside libsod (device buffers, the ctx stream);
  the production path.
* :class:`HostComm` -- the same exchanges staged through host memory over any object
  providing ``allgather``/``allreduce`` of numpy arrays (``FileHostComm`` over the
  stdlib :class:`FileStore` of one node; the CPU tests wrap a torch.distributed gloo group,
  ``tests/torch_comm.py``); used where RCCL is unavailable.

The bootstrap (RCCL unique id, barriers, max over ranks) needs nothing but the standard
library: :class:`FileStore`.

``run_sharded`` drives either one with the same code, so the multi-rank logic tested
with gloo on the CPU is the logic the GPUs run.
"""
from __future__ import annotations

import numpy as np


def shard_range(n, rank, world):
    return (n * rank) // world, (n * (rank + 1)) // world


class RcclComm:
    kind = "rccl"

    def __init__(self, ctx, world, rank, broadcast_bytes):
        """``broadcast_bytes(b or None) -> bytes`` distributes rank 0's RCCL unique id
        (any bootstrap channel: torch.distributed, MPI, a file)."""
        from . import _lib
        self.world, self.rank = world, rank
        uid = _lib.unique_id() if rank == 0 else None
        uid = broadcast_bytes(uid)
        ctx.comm_init(world, rank, uid)
        self._ctx = ctx

    def info(self):
        """The communicator as RCCL itself reports it: {"kind", "nranks", "rank"}."""
        n, r = self._ctx.comm_info()
        return {"kind": self.kind, "nranks": n, "rank": r}

    def gather_candidates(self, ctx):
        ctx.match_allgather()

    def reduce_histogram(self, ctx):
        ctx.hough_allreduce()


class HostComm:
    kind = "host"

    def __init__(self, world, rank, allgather, allreduce):
        """``allgather(arr) -> [arr_rank0, arr_rank1, ...]``;
        ``allreduce(arr, op) -> arr`` with op in {"sum", "min"}."""
        self.world, self.rank = world, rank
        self._allgather = allgather
        self._allreduce = allreduce

    def info(self):
        """{"kind": "host", "nranks", "rank"}: the host exchange's own world (no RCCL)."""
        return {"kind": self.kind, "nranks": self.world, "rank": self.rank}

    def gather_candidates(self, ctx):
        d1, idx, d2 = ctx.candidates()
        g1 = np.concatenate(self._allgather(d1))
        gi = np.concatenate(self._allgather(idx))
        g2 = np.concatenate(self._allgather(d2))
        ctx.merge_candidates(g1, gi, g2)

    def reduce_histogram(self, ctx):
        cnt, fst = ctx.hough_partial()
        cnt = self._allreduce(cnt.astype(np.int64), "sum").astype(np.uint32)
        fst = self._allreduce(fst.astype(np.int64), "min").astype(np.uint32)
        ctx.set_hough_partial(cnt, fst)


def _store_file(name):
    """A name a FileStore writes: ``gen``, ``<32 hex>_<key>``, ``.<name>.<rank>.tmp``, or one
    of its own keys (join / ready / broadcast / all-gather / done) under any hex generation
    or none (the files of a crashed run of an older format)."""
    import re
    return bool(name == "gen" or re.fullmatch(r"[0-9a-f]{32}_.+", name)
                or re.fullmatch(r"\..+\.\d+\.tmp", name)
                or re.fullmatch(r"(?:[0-9a-f]+_)?(?:ready|join_\d+|done_\d+|b\d+|g\d+_\d+)", name))


class FileStore:
    """Rendezvous of the ranks of ONE node through a directory (stdlib only): the RCCL
    unique-id broadcast, barriers, all-gathers of small byte strings.  Keys are files
    written to a temporary name and renamed into place (atomic), readers poll.

    ``path``: ``$SOD_STORE_DIR`` when set, else ``$TMPDIR/sod_store_<run id>`` with the run
    id of the launcher (``TORCHELASTIC_RUN_ID``, which torchrun gives every rank of one
    job), else ``<MASTER_PORT>_<parent pid>`` (the ranks a launcher started share their
    parent; ranks started by mpirun / srun / by hand have none in common and must set
    ``SOD_STORE_DIR``).  Every rank registers at construction and waits up to
    ``join_timeout`` seconds for the others, so ranks that landed in different directories
    fail at once with the path they used, not after ``timeout``.  ``close()`` removes the
    directory once every rank is done with it.

    Generations: a run that crashed leaves its files behind, and a later run in the same
    directory must not read them (an old RCCL unique id or all-gather payload).  Rank 0 clears
    the directory, then publishes a fresh random generation id in ``gen``; every key of the
    run is prefixed by it.  A rank > 0 joins the generation it reads with a random nonce of its
    own and proceeds only when rank 0's ``<gen>_ready`` echoes that nonce -- which a file left
    by an earlier run cannot -- re-joining whenever ``gen`` changes (it may have read a stale
    one before rank 0 cleared it)."""

    def __init__(self, world, rank, path=None, timeout=600.0, join_timeout=60.0):
        import os
        import tempfile
        self.world, self.rank, self.timeout = world, rank, timeout
        self._own_dir = False
        if path is None:
            path = os.environ.get("SOD_STORE_DIR")
        if path is None:
            self._own_dir = True          # sod_store_<run id>: made for this run, removed whole
            run = os.environ.get("TORCHELASTIC_RUN_ID")
            if not run or run == "none":
                run = "%s_%d" % (os.environ.get("MASTER_PORT", "0"), os.getppid())
            path = os.path.join(tempfile.gettempdir(), "sod_store_%s" % run)
        self.path = path
        os.makedirs(path, exist_ok=True)
        self._seq = 0
        self.gen = ""
        if world > 1:
            try:
                self._join(join_timeout)
            except TimeoutError as e:
                raise TimeoutError(
                    "FileStore: rank %d of %d: %s in %s within %.0f s -- ranks not started by "
                    "one launcher must share a directory: set SOD_STORE_DIR"
                    % (rank, world, e, path, join_timeout)) from None

    def _join(self, join_timeout):
        import json
        import os
        import time
        import uuid
        t0 = time.perf_counter()
        if self.rank == 0:
            for name in os.listdir(self.path):   # an earlier run's leftovers -- only files a
                if _store_file(name):             # store writes (the path may be shared)
                    try:
                        os.remove(os.path.join(self.path, name))
                    except OSError:
                        pass
            self.gen = uuid.uuid4().hex
            self._put("gen", self.gen.encode())
            nonces = {}
            for r in range(1, self.world):
                nonces[r] = self._wait("%s_join_%d" % (self.gen, r), t0, join_timeout,
                                       "found no rank %d" % r).decode()
            self._put("%s_ready" % self.gen, json.dumps(nonces).encode())
            return
        mine = uuid.uuid4().hex
        gen = None
        spin = 0
        while True:
            if time.perf_counter() - t0 > join_timeout:
                raise TimeoutError("found no rank 0 (generation %s)" % gen)
            g = self._read("gen")
            if g is not None and g.decode() != gen:
                gen = g.decode()
                self._put("%s_join_%d" % (gen, self.rank), mine.encode())
            if gen is not None:
                ready = self._read("%s_ready" % gen)
                if ready is not None and json.loads(ready.decode()).get(str(self.rank)) == mine:
                    self.gen = gen
                    return
            spin += 1
            if spin > 200:
                time.sleep(1e-4)

    def _put(self, name, data):
        import os
        tmp = os.path.join(self.path, ".%s.%d.tmp" % (name, self.rank))
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, os.path.join(self.path, name))

    def _read(self, name):
        try:
            with open(self._file_raw(name), "rb") as fh:
                return fh.read()
        except OSError:
            return None

    def _wait(self, name, t0, limit, what):
        import time
        spin = 0
        while True:
            d = self._read(name)
            if d is not None:
                return d
            if time.perf_counter() - t0 > limit:
                raise TimeoutError(what)
            spin += 1
            if spin > 200:
                time.sleep(1e-4)

    def _file_raw(self, name):
        import os
        return os.path.join(self.path, name)

    def _file(self, key):
        import os
        return os.path.join(self.path, "%s_%s" % (self.gen, key))

    def set(self, key, data):
        self._put("%s_%s" % (self.gen, key), data)

    def get(self, key):
        import os
        import time
        f = self._file(key)
        t0 = time.perf_counter()
        spin = 0
        while not os.path.exists(f):
            spin += 1
            if spin > 200:              # tight for ~the first ms (barriers in timed regions)
                time.sleep(1e-4)
            if time.perf_counter() - t0 > self.timeout:
                raise TimeoutError("FileStore: rank %d waited %.0f s for %s"
                                   % (self.rank, self.timeout, key))
        with open(f, "rb") as fh:
            return fh.read()

    def allgather_bytes(self, data):
        k = self._seq
        self._seq += 1
        self.set("g%d_%d" % (k, self.rank), data)
        return [self.get("g%d_%d" % (k, r)) for r in range(self.world)]

    def barrier(self):
        self.allgather_bytes(b"")

    def broadcast_bytes(self, data):
        """rank 0's bytes on every rank (``data`` is ignored elsewhere)."""
        k = self._seq
        self._seq += 1
        if self.rank == 0:
            self.set("b%d" % k, data)
            return data
        return self.get("b%d" % k)

    def max(self, x):
        import struct
        return max(struct.unpack("<d", b)[0] for b in self.allgather_bytes(struct.pack("<d", x)))

    def sum(self, x):
        import struct
        return sum(struct.unpack("<d", b)[0] for b in self.allgather_bytes(struct.pack("<d", x)))

    def close(self):
        import shutil
        self.barrier()                   # every rank has read everything it will read
        self.set("done_%d" % self.rank, b"")
        if self.rank == 0:
            import os
            for r in range(self.world):
                self.get("done_%d" % r)
            if self._own_dir:
                shutil.rmtree(self.path, ignore_errors=True)
            else:                        # a caller's directory: only the store's own files,
                for name in os.listdir(self.path):   # then the directory if that emptied it
                    if _store_file(name):
                        try:
                            os.remove(os.path.join(self.path, name))
                        except OSError:
                            pass
                try:
                    os.rmdir(self.path)
                except OSError:
                    pass


class FileHostComm(HostComm):
    """HostComm over a :class:`FileStore` (no torch, no MPI): the host-staged exchanges of
    ranks that cannot use RCCL (e.g. several ranks sharing one GPU)."""

    def __init__(self, store):
        def allgather(a):
            a = np.ascontiguousarray(a)
            return [np.frombuffer(b, a.dtype).reshape(a.shape)
                    for b in store.allgather_bytes(a.tobytes())]

        def allreduce(a, op):
            parts = allgather(a)
            out = parts[0].copy()
            for p in parts[1:]:
                out = out + p if op == "sum" else np.minimum(out, p)
            return out

        super().__init__(store.world, store.rank, allgather, allreduce)


def run_sharded(ctx, comm, shard, query_shape, bins, ratio=0.75, vote_threshold=5,
                affine_threshold=4, x_factor=128.0, y_factor=128.0, run_affine=True):
    """One query image over the sharded database.  ``shard`` = (lo, hi) global rows held
    by this rank's ``ctx``.  Leaves the results in ``ctx`` (match_result, valid_result,
    affine_result are then identical on every rank)."""
    ctx.match()
    comm.gather_candidates(ctx)
    ctx.ratio(ratio)
    ctx.hough(query_shape, bins, own=shard)
    comm.reduce_histogram(ctx)
    ctx.select(vote_threshold)
    if run_affine:
        ctx.affine((query_shape[1], query_shape[0]), x_factor, y_factor, affine_threshold)
