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
