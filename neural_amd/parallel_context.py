"""Tensor-parallel communicator: the reference's parallel_context (neural_speed/core/parallel_context.h:28-52,
parallel_context.cpp:19-137, oneCCL over MPI or a same-host SHM all-reduce) re-hosted on torch.distributed.

One process per GPU; backend "nccl" is RCCL on ROCm (point-to-point xGMI between the 8 MI355X of a node), "gloo"
on CPU.  Counts are element counts of the tensors passed (the reference passes byte counts as element counts at
ne_layers.c:5474 / llama.cpp:185 -- not replicated).
"""
import os

import torch
import torch.distributed as dist


class ParallelContext:
    """init_parallel_context() / get_tp_size / get_tp_rank / is_master / barrier / broadcast / alltoall / reduce_add"""

    def __init__(self, backend=None, group=None, device=None):
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            kw = {"device_id": torch.device("cuda", device)} if (backend == "nccl" and device is not None) else {}
            dist.init_process_group(backend, **kw)
        self.group = group

    def get_tp_size(self):
        return dist.get_world_size(self.group)

    def get_tp_rank(self):
        return dist.get_rank(self.group)

    def is_master(self):
        return self.get_tp_rank() == 0

    def barrier(self):
        dist.barrier(self.group)

    def broadcast(self, buffer, root=0):
        dist.broadcast(buffer, root, group=self.group)
        return buffer

    def alltoall(self, send, recv):
        dist.all_to_all_single(recv, send, group=self.group)
        return recv

    def reduce_add(self, send, recv=None):
        """sum over ranks (parallel_context.cpp:47-57); in place when recv is None or is send."""
        if recv is not None and recv is not send:
            recv.copy_(send)
            send = recv
        dist.all_reduce(send, op=dist.ReduceOp.SUM, group=self.group)
        return send

    def max_over_ranks(self, value):
        t = torch.tensor([float(value)], dtype=torch.float64,
                         device="cuda" if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def destroy(self):
        if dist.is_initialized():
            dist.destroy_process_group()

    def all_gather_cols(self, local, sizes):
        """concatenate column shards [M, n_r] of every rank into [M, sum n_r] (column-parallel output gather)."""
        world = self.get_tp_size()
        parts = [torch.empty((local.shape[0], s), dtype=local.dtype, device=local.device) for s in sizes]
        if len(set(sizes)) == 1:
            dist.all_gather(parts, local.contiguous(), group=self.group)
        else:  # uneven shards: pad to the max width
            w = max(sizes)
            pad = torch.zeros((local.shape[0], w), dtype=local.dtype, device=local.device)
            pad[:, :local.shape[1]] = local
            full = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(full, pad, group=self.group)
            parts = [f[:, :s] for f, s in zip(full, sizes)]
        return torch.cat(parts, dim=1)
