"""Communicator: the engine's replacement for ``mpisppy.MPI`` (MPI.py:3-82).

One process per GPU; collectives go through ``torch.distributed`` — backend
"nccl" (= RCCL over xGMI on ROCm) when tensors live on the GPU, "gloo" for the
CPU multi-process tests.  Without an initialised process group the
communicator is a single-rank stand-in (the reference's ``_MockMPIComm``,
MPI.py:19-82: rank 0, size 1, Allreduce copies).

Only what the PH path needs: an in-place SUM allreduce of one fused fp64
buffer per PH step (replacing the per-tree-node ``comms[ndn].Allreduce`` of
phbase.py:83-87 and the scalar reductions of phbase.py:341 and
spopt.py:341-466), barrier, and host-object gather/broadcast for setup checks.
"""
import os

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, group=None):
        self.group = group
        if group is not None or (dist.is_available() and dist.is_initialized()):
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank = 0
            self.size = 1
            self.backend = None

    # mpi4py-style accessors used by the reference API
    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def _reduce(self, t, op):
        if self.size == 1:
            return t
        if t.is_cuda and self.backend != "nccl":
            # gloo over device tensors (several ranks sharing one GPU, the
            # multi-rank GPU tests): staged through the host -- the read-back
            # waits on the current stream for the kernels that produced t, and
            # the result is written back in that stream's order
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=self.group)
        return t

    def allreduce_(self, t):
        """In-place SUM over ranks of a torch tensor (no-op on one rank)."""
        return self._reduce(t, dist.ReduceOp.SUM)

    def allreduce_max_(self, t):
        return self._reduce(t, dist.ReduceOp.MAX)

    def Barrier(self):
        if self.size > 1:
            dist.barrier(group=self.group)

    barrier = Barrier

    def allgather_object(self, obj):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def gather(self, obj, root=0):
        allv = self.allgather_object(obj)
        return allv if self.rank == root else None

    def bcast(self, obj, root=0):
        if self.size == 1:
            return obj
        lst = [obj]
        # broadcast_object_list takes a GLOBAL source rank
        src = dist.get_global_rank(self.group, root) if self.group is not None else root
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def allreduce_np(self, arr, op="sum"):
        """Allreduce of a small host array (write ids, flags): on a GPU tensor
        for RCCL groups, on the host for gloo.  Returns a new numpy array."""
        import numpy as np
        a = np.asarray(arr)
        if self.size == 1:
            return a.copy()
        t = torch.as_tensor(a.copy())
        if self.backend == "nccl":
            t = t.to("cuda")
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop, group=self.group)
        return t.cpu().numpy()

    def Split(self, color, key):
        """mpi4py's ``Comm.Split``: ranks with the same color form a new
        communicator, ordered by key.  Every rank of this communicator must
        call it (torch.distributed creates each group collectively)."""
        if self.size == 1:
            return Comm(self.group)
        entries = self.allgather_object((int(color), int(key), dist.get_rank()))
        mine = None
        for c in sorted({e[0] for e in entries}):
            members = [g for (cc, k, g) in sorted((e for e in entries if e[0] == c), key=lambda e: (e[1], e[2]))]
            grp = dist.new_group(ranks=members)
            if c == int(color):
                mine = grp
        return Comm(mine)


def world():
    return Comm()


def init_from_env(device_type="cuda"):
    """Initialise torch.distributed from torchrun's env vars (RANK/WORLD_SIZE/...).
    Backend "nccl" (RCCL) for GPU tensors, "gloo" for CPU.  Returns Comm."""
    if dist.is_initialized():
        return Comm()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if device_type == "cuda" else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend=backend)
    return Comm()
