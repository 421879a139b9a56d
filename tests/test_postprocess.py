"""SURVEY §8(f) row 1 -- post-processing (PostProcessing.py:4-112, main.py:159-168).

CPU: the oracle restatement against golden vectors made by the reference's own
PostProcessing functions (tests/golden/make_golden.py, ``post_*``), bit for bit, and the
pure-host drop-in helpers (``dfs``, ``find_max_orientation``, ``get_final_pose``).
GPU: the device pass (bitmask relations + DFS in the reference's order) against the same
goldens and the oracle, through the C ABI and through ``Main.post_process``."""
import math

import numpy as np
import pytest

from conftest import golden
from oracle import oracle as orc
from sift_based_od_amd import _lib, postprocessing as pp
from sift_based_od_amd.posebin import PoseBin

POST = ["post_edge", "post_small", "post_medium", "post_chain"]
E2E = ["c1_b15", "planted_b15", "planted_b12", "edge_b15", "edge_b6"]


def _bins(means):
    return [PoseBin((0, 0, 0, 0), (float(r[4]), float(r[5])), 1, [],
                    (float(r[0]), float(r[1]), float(r[2]), float(r[3]))) for r in means]


def _flat(clusters):
    return np.array([k for c in clusters for k in c], np.int64)


def _fp_rows(fp):
    return np.array([[p[0][0], p[0][1], p[1], p[2], p[3][0], p[3][1]] for p in fp],
                    np.float64).reshape(-1, 6)


@pytest.mark.parametrize("name", POST)
def test_oracle_post_golden(name):
    g = golden(name)
    r = orc.post_process(g["means"])
    assert np.array_equal(_flat(r["pose_cluster"]), g["pos_members"])
    assert np.array_equal(np.cumsum([0] + [len(c) for c in r["pose_cluster"]]), g["pos_off"])
    assert np.array_equal(_flat([k for oc in r["orientation_cluster"] for k in oc]),
                          g["ori_members"])
    assert np.array_equal(np.array(r["final_orientation"]).view(np.uint64),
                          g["final_orientation"].view(np.uint64))
    assert np.array_equal(_fp_rows(r["final_pose"]).view(np.uint64), g["final_pose"].view(np.uint64))


@pytest.mark.parametrize("name", E2E)
def test_oracle_post_on_pipeline_survivors(name):
    """main.py's final_pose on the reference's surviving bins (their PoseBin means)."""
    g = golden(name)
    if "final_pose" not in g:
        pytest.skip("no final pose recorded")
    means = g["valid_means"][g["surv_index"]]
    r = orc.post_process(means)
    assert np.array_equal(_fp_rows(r["final_pose"]).view(np.uint64), g["final_pose"].view(np.uint64))


@pytest.mark.parametrize("name", POST)
def test_host_helpers_golden(name):
    """dfs / find_max_orientation / get_final_pose drop-ins on PoseBin objects, fed the
    reference's clusters."""
    g = golden(name)
    bins = _bins(g["means"])
    off, mem = g["pos_off"], g["pos_members"]
    pc = [[bins[k] for k in mem[off[c]:off[c + 1]]] for c in range(len(off) - 1)]
    oc = []
    for c in range(len(off) - 1):
        lo, hi = g["ori_pos_off"][c], g["ori_pos_off"][c + 1]
        oc.append([[bins[k] for k in g["ori_members"][g["ori_off"][o]:g["ori_off"][o + 1]]]
                   for o in range(lo, hi)])
    fo = pp.find_max_orientation(oc)
    assert np.array_equal(np.array(fo, np.float64).view(np.uint64),
                          g["final_orientation"].view(np.uint64))
    fp = pp.get_final_pose(pc, fo)
    assert np.array_equal(_fp_rows(fp).view(np.uint64), g["final_pose"].view(np.uint64))
    # dfs over the reference's own adjacency construction reproduces the clusters
    n = len(bins)
    adj = {b: [] for b in range(n)}
    for b in range(n):
        for a in range(b):
            if orc.position_close(tuple(g["means"][a]), tuple(g["means"][b])):
                adj[b].append(a)
                adj[a].append(b)
    seen, got = set(), []
    for i in range(n):
        if i not in seen:
            got.append(pp.dfs(i, seen, adj, [], list(range(n))))
    assert np.array_equal(_flat(got), mem)


@pytest.mark.gpu
@pytest.mark.parametrize("name", POST)
def test_device_post_batch_golden(ctx, name):
    g = golden(name)
    r = ctx.post_batch(g["means"])
    for k in ("pos_off", "pos_members", "ori_pos_off", "ori_off", "ori_members"):
        assert np.array_equal(r[k], g[k]), k
    assert np.array_equal(r["final_orientation"].view(np.uint64), g["final_orientation"].view(np.uint64))
    assert np.array_equal(r["final_pose"].view(np.uint64), g["final_pose"].view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(0, 0), (1, 1), (40, 4), (64, 5), (65, 2), (1500, 3)])
def test_device_post_batch_vs_oracle(ctx, n, seed):
    rng = np.random.default_rng(seed)
    c = rng.integers(0, max(1, n // 20), n)
    cx, cy = rng.uniform(0, 20000, 1000), rng.uniform(0, 15000, 1000)
    ca = rng.uniform(0, 2 * math.pi, 1000)
    s = 2.0 ** rng.integers(-1, 2, n)
    w, h = rng.choice([1500.0, 900.0], n), rng.uniform(800, 1200, n)
    means = np.stack([cx[c] + rng.normal(0, 300, n), cy[c] + rng.normal(0, 300, n),
                      ca[c] + np.radians(rng.normal(0, 1.0, n)), s, w, h], 1).reshape(-1, 6)
    r = ctx.post_batch(means)
    o = orc.post_process(means)
    assert np.array_equal(r["pos_members"], _flat(o["pose_cluster"]))
    assert np.array_equal(r["ori_members"],
                          _flat([k for oc in o["orientation_cluster"] for k in oc]))
    assert np.array_equal(r["final_pose"], _fp_rows(o["final_pose"]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_b15", "planted_b15", "planted_b12"])
def test_pipeline_postprocess_golden(ctx, name, trig):
    """Full device pipeline then post-processing over the survivors == main.py's final
    pose bit for bit (with the device's glibc cos / sin even without the host's redo of the
    survivors' x / y means, sod_set_post_exact(0))."""
    from helpers import kp
    g = golden(name)
    ctx.set_keypoints(kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
    ctx.upload_db(g["db_des"])
    ctx.upload_queries(g["q_des"], kp(g, "q_"))
    ctx.pipeline(tuple(int(v) for v in g["shape"]), int(g["bins"]))
    r = ctx.postprocess_getter()                # sod_postprocess
    assert np.array_equal(r["bin_index"], g["surv_index"])
    f = ctx.postprocess()                       # the one-transfer form: the same outputs
    for k in r:
        assert np.array_equal(f[k], r[k]), k
    # the survivors' x / y means redone with glibc (sod_set_post_exact, default): main.py's
    # final pose bit for bit
    assert np.array_equal(r["final_pose"].view(np.uint64),
                          np.asarray(g["final_pose"], np.float64).view(np.uint64))
    ctx.set_post_exact(False)   # the device means alone
    r = ctx.postprocess()
    ctx.set_post_exact(True)
    if ctx.trig_exact():   # device glibc cos / sin: already main.py's bit for bit
        assert np.array_equal(r["final_pose"].view(np.uint64),
                              np.asarray(g["final_pose"], np.float64).view(np.uint64))
    np.testing.assert_allclose(r["final_pose"], g["final_pose"], rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["edge_b15", "edge_b6"])
def test_stage_api_postprocess_golden(ctx, name, trig):
    """Stage entry points on the golden matches (hough -> select -> affine), then the
    device post-processing over the survivors -> main.py's final_pose."""
    from helpers import kp
    g = golden(name)
    r = ctx
    shape = tuple(int(v) for v in g["shape"])
    r.set_keypoints(kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
    r.upload_queries(None, kp(g, "q_"))
    idx1 = np.zeros(len(g["q_x"]), np.int32)
    idx1[g["match_q"]] = g["match_m"]
    good = np.zeros(len(g["q_x"]), bool)
    good[g["match_q"]] = True
    r.set_matches(idx1, good)
    r.hough(shape, int(g["bins"]))
    r.select(5)
    r.affine((shape[1], shape[0]), 128.0, 128.0, 4)
    res = r.postprocess()
    assert np.array_equal(res["final_pose"].view(np.uint64),
                          np.asarray(g["final_pose"], np.float64).view(np.uint64))
