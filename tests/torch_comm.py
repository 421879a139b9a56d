"""HostComm over a torch.distributed process group (gloo): the CPU tests' adapter for the
product's host-staged exchange (``sharded.HostComm``).  Test code only -- the product
bootstraps without PyTorch (``sharded.FileStore``)."""
import numpy as np

from sift_based_od_amd.sharded import HostComm


class TorchHostComm(HostComm):
    """HostComm over a torch.distributed process group (gloo): a test adapter."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self._t, self._d, self._g = torch, dist, group

        def allgather(a):
            t = torch.from_numpy(np.ascontiguousarray(a))
            out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
            dist.all_gather(out, t, group=group)
            return [o.numpy() for o in out]

        def allreduce(a, op):
            t = torch.from_numpy(np.ascontiguousarray(a))
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MIN,
                            group=group)
            return t.numpy()

        super().__init__(dist.get_world_size(group), dist.get_rank(group), allgather, allreduce)
