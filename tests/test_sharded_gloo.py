"""Multi-rank path on the CPU: the product's ``run_sharded`` + ``TorchHostComm`` (tests/torch_comm.py) over a
real torch.distributed gloo group (world_size 2), with the oracle test double standing
in for the device.  The sharded result must equal the single-rank result bit for bit
(global top-2 merge before the ratio test; partial histograms reduced
with sum/min)."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    sys.path.insert(0, os.path.dirname(HERE))
    import sod_pkg
    sod_pkg.load()
    from sift_based_od_amd import synthetic
    db = synthetic.make_database(4, 150, seed=21)
    qs = synthetic.make_queries(400, seed=22, db_seed=21, kp_per_image=150, planted_frac=0.5,
                                decoy_frac=0.1)
    return db, qs


def _worker(rank, world, port, outdir, bins):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import sod_pkg
    sod_pkg.load()
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    from fake_ctx import OracleCtx
    from sift_based_od_amd.sharded import run_sharded, shard_range
    from torch_comm import TorchHostComm
    db, qs = _case()
    lo, hi = shard_range(len(db), rank, world)
    ctx = OracleCtx(db, lo, hi, qs.des, qs.kp)
    run_sharded(ctx, TorchHostComm(), (lo, hi), qs.shape, bins, 0.75, 5, 4, 128.0, 128.0, True)
    idx1, d1, d2, good = ctx.match_result()
    v = ctx.valid_result()
    surv = np.array([r["survived"] for r in ctx.affine_result()], bool)
    np.savez(os.path.join(outdir, "r%d.npz" % rank), idx1=idx1, d1=d1, d2=d2, good=good,
             keys=v["keys"], votes=v["votes"], off=v["offsets"], mem=v["members"], surv=surv)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bins", [(2, 15), (3, (12, 12, 8, 6))])
def test_sharded_equals_single_rank(tmp_path, world, bins):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), bins), nprocs=world, join=True)
    sys.path.insert(0, HERE)
    from fake_ctx import OracleCtx
    from sift_based_od_amd.sharded import HostComm, run_sharded
    db, qs = _case()
    ref = OracleCtx(db, 0, len(db), qs.des, qs.kp)
    single = HostComm(1, 0, lambda a: [a], lambda a, op: a)
    run_sharded(ref, single, (0, len(db)), qs.shape, bins, 0.75, 5, 4, 128.0, 128.0, True)
    idx1, d1, d2, good = ref.match_result()
    v = ref.valid_result()
    surv = np.array([r["survived"] for r in ref.affine_result()], bool)
    assert len(v["keys"]) > 0 and surv.any()
    for r in range(world):
        z = np.load(tmp_path / ("r%d.npz" % r))
        assert np.array_equal(z["idx1"], idx1) and np.array_equal(z["good"], good)
        assert np.array_equal(z["d1"], d1) and np.array_equal(z["d2"], d2)
        assert np.array_equal(z["keys"], v["keys"]) and np.array_equal(z["votes"], v["votes"])
        assert np.array_equal(z["off"], v["offsets"]) and np.array_equal(z["mem"], v["members"])
        assert np.array_equal(z["surv"], surv)


def _file_worker(rank, world, store_path, outdir, bins):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import sod_pkg
    sod_pkg.load()
    from fake_ctx import OracleCtx
    from sift_based_od_amd.sharded import FileHostComm, FileStore, run_sharded, shard_range
    store = FileStore(world, rank, path=store_path, timeout=120)
    # the bootstrap primitives bench.py uses: unique-id broadcast, barrier, max / sum
    uid = store.broadcast_bytes(b"uid-from-rank-0" if rank == 0 else None)
    assert uid == b"uid-from-rank-0"
    store.barrier()
    assert store.max(float(rank)) == world - 1
    assert store.sum(1.0) == world
    db, qs = _case()
    lo, hi = shard_range(len(db), rank, world)
    ctx = OracleCtx(db, lo, hi, qs.des, qs.kp)
    run_sharded(ctx, FileHostComm(store), (lo, hi), qs.shape, bins, 0.75, 5, 4, 128.0, 128.0, True)
    idx1, d1, d2, good = ctx.match_result()
    v = ctx.valid_result()
    surv = np.array([r["survived"] for r in ctx.affine_result()], bool)
    np.savez(os.path.join(outdir, "f%d.npz" % rank), idx1=idx1, d1=d1, d2=d2, good=good,
             keys=v["keys"], votes=v["votes"], off=v["offsets"], mem=v["members"], surv=surv)
    store.close()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_over_file_store_equals_single_rank(tmp_path, world):
    """bench.py's torch-free multi-rank plumbing: FileStore bootstrap + FileHostComm
    exchange between real processes, equal to the single-rank result bit for bit; the
    store directory is gone after close()."""
    import multiprocessing as mp
    bins = 15
    store_path = str(tmp_path / "store")
    ctxm = mp.get_context("spawn")
    procs = [ctxm.Process(target=_file_worker, args=(r, world, store_path, str(tmp_path), bins))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert not os.path.exists(store_path)
    sys.path.insert(0, HERE)
    from fake_ctx import OracleCtx
    from sift_based_od_amd.sharded import HostComm, run_sharded
    db, qs = _case()
    ref = OracleCtx(db, 0, len(db), qs.des, qs.kp)
    run_sharded(ref, HostComm(1, 0, lambda a: [a], lambda a, op: a), (0, len(db)), qs.shape,
                bins, 0.75, 5, 4, 128.0, 128.0, True)
    idx1, _, _, good = ref.match_result()
    v = ref.valid_result()
    for r in range(world):
        z = np.load(tmp_path / ("f%d.npz" % r))
        assert np.array_equal(z["idx1"], idx1) and np.array_equal(z["good"], good)
        assert np.array_equal(z["keys"], v["keys"]) and np.array_equal(z["mem"], v["members"])


def test_single_rank_double_matches_oracle_pipeline():
    """The test double itself agrees with the oracle's end-to-end restatement."""
    sys.path.insert(0, HERE)
    from fake_ctx import OracleCtx
    from oracle import oracle as orc
    from sift_based_od_amd.sharded import HostComm, run_sharded
    db, qs = _case()
    ref = OracleCtx(db, 0, len(db), qs.des, qs.kp)
    run_sharded(ref, HostComm(1, 0, lambda a: [a], lambda a, op: a), (0, len(db)), qs.shape,
                15, 0.75, 5, 4, 128.0, 128.0, True)
    dbkp = {"x": db.kp.x, "y": db.kp.y, "angle": db.kp.angle, "octave": db.kp.octave,
            "img": db.img}
    qkp = {"x": qs.kp.x, "y": qs.kp.y, "angle": qs.kp.angle, "octave": qs.kp.octave}
    out = orc.run_pipeline(qs.des, qkp, db.des, dbkp, {"centroid": db.centroid, "size": db.size},
                           15, qs.shape)
    v = ref.valid_result()
    assert [tuple(k) for k in v["keys"]] == [b.pose for b in out["valid"]]
    assert list(v["votes"]) == [b.votes for b in out["valid"]]
    assert [r["survived"] for r in ref.affine_result()] == [r["survived"] for r in out["affine"]]


def test_shard_range_covers_rows():
    sys.path.insert(0, os.path.dirname(HERE))
    from sift_based_od_amd.sharded import shard_range
    for n in (1, 7, 1000, 8_000_000):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, i, w) for i in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[i][1] == r[i + 1][0] for i in range(w - 1))


def test_file_store_fails_fast_without_shared_dir(tmp_path, monkeypatch):
    """Ranks that do not share a store directory (no common launcher, no SOD_STORE_DIR) fail
    at construction with the path they used, not after the exchange timeout."""
    import time
    sys.path.insert(0, os.path.dirname(HERE))
    import sod_pkg
    sod_pkg.load()
    from sift_based_od_amd.sharded import FileStore
    t0 = time.perf_counter()
    with pytest.raises(TimeoutError, match="SOD_STORE_DIR"):
        FileStore(2, 1, path=str(tmp_path / "alone"), timeout=600, join_timeout=0.5)
    assert time.perf_counter() - t0 < 30
    # the directory choice: explicit env first, then the launcher's run id
    monkeypatch.setenv("SOD_STORE_DIR", str(tmp_path / "env"))
    assert FileStore(1, 0).path == str(tmp_path / "env")
    monkeypatch.delenv("SOD_STORE_DIR")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job42_%d" % os.getpid())
    st = FileStore(1, 0)
    assert st.path.endswith("sod_store_job42_%d" % os.getpid())
    st.close()
    assert not os.path.exists(st.path)


def _store_rank(path, world, rank, q):
    sys.path.insert(0, os.path.dirname(HERE))
    import sod_pkg
    sod_pkg.load()
    from sift_based_od_amd.sharded import FileStore
    st = FileStore(world, rank, path=path, timeout=60, join_timeout=30)
    got = st.broadcast_bytes(b"fresh-%d" % os.getpid() if rank == 0 else b"")
    parts = st.allgather_bytes(b"r%d" % rank)
    q.put((rank, got, parts))
    st.close()


def test_file_store_ignores_an_unclosed_runs_files(tmp_path):
    """a crashed run's files (its join marks, an RCCL-id broadcast, all-gather
    payloads, an old generation and ready mark) stay in the directory; a new run there must
    neither join on them nor read their payloads."""
    import json
    import multiprocessing as mp
    path = tmp_path / "store"
    path.mkdir()
    old = "deadbeef"
    (path / "gen").write_bytes(old.encode())
    (path / ("%s_ready" % old)).write_bytes(json.dumps({"1": "x"}).encode())
    for name, data in [("join_0", b""), ("join_1", b""), ("b0", b"stale"), ("g1_0", b"stale"),
                       ("g1_1", b"stale"), ("%s_b0" % old, b"stale"), ("%s_g1_0" % old, b"stale"),
                       ("%s_g1_1" % old, b"stale"), ("%s_join_1" % old, b"x")]:
        (path / name).write_bytes(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # rank 1 first: it reads the stale generation before rank 0 clears it
    procs = [ctx.Process(target=_store_rank, args=(str(path), 2, r, q)) for r in (1, 0)]
    procs[0].start()
    import time
    time.sleep(1.0)
    procs[1].start()
    out = dict((r, (g, p)) for r, g, p in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert out[0][0].startswith(b"fresh-") and out[1][0] == out[0][0]
    assert out[0][1] == out[1][1] == [b"r0", b"r1"]
    assert not path.exists()   # close() removed the directory


def test_file_store_keeps_unrelated_files(tmp_path):
    """SOD_STORE_DIR may be a shared directory; a run there removes only the
    files a store writes (its own and a crashed run's), never the directory's other files."""
    import multiprocessing as mp
    path = tmp_path / "shared"
    path.mkdir()
    for name in ("notes.txt", "gen2", "abc_def", "data.npz"):
        (path / name).write_bytes(b"keep")
    (path / "join_1").write_bytes(b"")                  # a crashed run's key: removed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_store_rank, args=(str(path), 2, r, q)) for r in (0, 1)]
    for p in procs:
        p.start()
    out = dict((r, (g, p)) for r, g, p in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert out[0][1] == out[1][1] == [b"r0", b"r1"]
    assert sorted(os.listdir(path)) == ["abc_def", "data.npz", "gen2", "notes.txt"]


def test_torch_host_comm_removed():
    """TorchHostComm left the exports in round 4 and its deprecated alias in round 6: the name
    no longer resolves (FileHostComm, or a HostComm over the caller's own collectives)."""
    import sift_based_od_amd as pkg
    from sift_based_od_amd import sharded
    for mod in (pkg, sharded):
        with pytest.raises(AttributeError):
            getattr(mod, "TorchHostComm")
