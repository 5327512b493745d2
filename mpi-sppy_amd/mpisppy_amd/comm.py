"""Communicator over ``torch.distributed`` (RCCL on GPU, gloo on CPU).

Replaces the mpi4py communicator the reference passes around
(``spbase.py:78-85``).  One rank per GPU.  The per-tree-node
sub-communicators of the reference (``spbase.py:311-350``) are not needed:
per-node sums are packed into one dense buffer in which ranks that do not
hold a node contribute zeros, so a single allreduce over the cylinder group
equals the reference's per-node ``Split`` reductions.
"""
import torch
import torch.distributed as dist


class Comm:
    """Thin wrapper: rank/size/allreduce/barrier/gather_object."""

    def __init__(self, group=None):
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        if self.distributed:
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank = 0
            self.size = 1
            self.backend = None

    @classmethod
    def wrap(cls, mpicomm):
        if isinstance(mpicomm, Comm):
            return mpicomm
        return cls(mpicomm)

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def allreduce_(self, t, op="sum"):
        """In-place allreduce of a tensor (device tensors go over RCCL)."""
        if self.size == 1:
            return t
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        if self.backend == "gloo" and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=rop, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=rop, group=self.group)
        return t

    def allreduce_host(self, values, op="sum", dtype=torch.float64):
        """Allreduce a short list of host numbers; returns a list."""
        t = torch.tensor(values, dtype=dtype)
        if self.size > 1:
            if self.backend == "nccl":
                t = t.cuda()
            self.allreduce_(t, op)
        return t.cpu().tolist()

    def Barrier(self):
        if self.size > 1:
            dist.barrier(group=self.group)

    def allgather_object(self, obj):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def gather_object(self, obj, root=0):
        allv = self.allgather_object(obj)
        return allv if self.rank == root else None
