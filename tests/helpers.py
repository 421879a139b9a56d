"""Shared test helpers: fixture -> arrays, oracle adapters, in-process communicator."""
import threading

import numpy as np

from sift_based_od_amd.database import Keypoints


def kp(g, prefix):
    return Keypoints(g[prefix + "x"], g[prefix + "y"], g[prefix + "angle"], g[prefix + "octave"])


def kp_dict(k, img=None):
    d = {"x": k.x, "y": k.y, "angle": k.angle, "octave": k.octave}
    if img is not None:
        d["img"] = img
    return d


def csr_lists(off, mem):
    return [list(mem[off[i]:off[i + 1]]) for i in range(len(off) - 1)]


class ThreadComm:
    """allgather / allreduce between threads of one process (test plumbing)."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world

    def for_rank(self, r):
        from sift_based_od_amd.sharded import HostComm

        def allgather(a):
            self.slots[r] = np.array(a)
            self.bar.wait()
            out = list(self.slots)
            self.bar.wait()
            return out

        def allreduce(a, op):
            parts = allgather(a)
            return (np.sum(parts, axis=0) if op == "sum" else np.min(parts, axis=0)).astype(a.dtype)

        return HostComm(self.world, r, allgather, allreduce)


def oracle_inputs(db, qs_kp):
    """Oracle-side dicts for a SiftDatabase and a query Keypoints SoA."""
    dbkp = {"x": db.kp.x, "y": db.kp.y, "angle": db.kp.angle, "octave": db.kp.octave,
            "img": db.img}
    qkp = {"x": qs_kp.x, "y": qs_kp.y, "angle": qs_kp.angle, "octave": qs_kp.octave}
    images = {"centroid": db.centroid, "size": db.size}
    return dbkp, qkp, images


def assert_stages_equal_oracle(valid, aff, ref_table, ref_valid, ref_aff, q_offset=0,
                               bins_all=None, post=None, affine_atol=1e-4):
    """Device results of the stages after the matcher against the oracle's: the full bin
    table in first-touch order (``bins_all`` = Context.all_bins(), optional), valid bins,
    member lists (device query index - ``q_offset`` = oracle query index), PoseBin means
    (1e-12 relative), affine survivors / votes / kept members exactly, parameters within
    ``affine_atol`` (north_star), and, with ``post`` = Context.postprocess(), the
    post-processing final poses."""
    import numpy as np
    from oracle import oracle as orc

    if bins_all is not None:
        keys, votes = bins_all
        assert [tuple(int(v) for v in k) for k in keys] == list(ref_table.keys()), \
            "bin table (first-touch order) differs"
        assert list(votes) == [b.votes for b in ref_table.values()]
    assert [tuple(int(x) for x in k) for k in valid["keys"]] == [b.pose for b in ref_valid]
    assert list(valid["votes"]) == [b.votes for b in ref_valid]
    off, mem = valid["offsets"], valid["members"]
    for i, b in enumerate(ref_valid):
        assert [int(q) - q_offset for q in mem[off[i]:off[i + 1]]] == [q for q, _ in b.members]
    if ref_valid:
        ref_means = np.array([[b.centroid[0], b.centroid[1], b.angle, b.scale, b.img_size[0],
                               b.img_size[1]] for b in ref_valid])
        np.testing.assert_allclose(valid["means"], ref_means, rtol=1e-12, atol=1e-9)
    if aff is not None:
        assert [bool(s) for s in aff["survived"]] == [r["survived"] for r in ref_aff]
        for i in np.nonzero(aff["survived"])[0]:
            assert aff["votes"][i] == ref_aff[i]["votes"]
            np.testing.assert_allclose(aff["params"][i], ref_aff[i]["params"], rtol=0,
                                       atol=affine_atol)
            lo, hi = off[i], off[i + 1]
            kept = mem[lo:hi][aff["alive"][lo:hi]]
            assert [int(q) - q_offset for q in kept] == [q for q, _ in ref_aff[i]["members"]]
    if post is not None:
        ref = orc.post_process(valid["means"][post["bin_index"]])
        fp = np.array([[p[0][0], p[0][1], p[1], p[2], p[3][0], p[3][1]]
                       for p in ref["final_pose"]]).reshape(-1, 6)
        np.testing.assert_allclose(post["final_pose"], fp, rtol=1e-12, atol=1e-9)
