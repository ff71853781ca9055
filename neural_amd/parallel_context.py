"""Tensor-parallel communicator: Python face of the library's C-ABI parallel context (include/neural_amd.h,
csrc/parallel_context.hip), which replaces the reference's neural_speed/core/parallel_context.{h,cpp}
(init_parallel_context / get_tp_size / get_tp_rank / is_master / barrier / broadcast / alltoall / reduce_add).

One process per GPU.  Device tensors are reduced on the caller's current HIP stream (one-shot IPC all-reduce for small
messages, RCCL over xGMI for large ones); host tensors go through the reference's synchronous entry points.  Without a
GPU (transport="tcp") the rendezvous sockets carry host tensors, which is how the CPU tests run the N>1 logic.
Element counts, not byte counts (the reference passes bytes as elements at ne_layers.c:5474 -- not replicated).
"""
import ctypes as C
import os

from ._lib import lib


class ParallelContext:
    def __init__(self, transport=None, keep_device=True):
        """transport: None (GPU when present) or "tcp" (host tensors over the rendezvous sockets, no GPU).
        keep_device: use the HIP device the caller selected (torch.cuda.set_device) instead of LOCAL_RANK % devices."""
        if transport:
            os.environ["NAD_PC_TRANSPORT"] = transport
        if keep_device:
            os.environ["NAD_PC_KEEP_DEVICE"] = "1"
        L = self.L = lib()
        self.p = L.init_parallel_context()
        if not self.p:
            raise RuntimeError("init_parallel_context failed (see stderr)")

    def get_tp_size(self):
        return self.L.get_tp_size(self.p)

    def get_tp_rank(self):
        return self.L.get_tp_rank(self.p)

    def is_master(self):
        return bool(self.L.is_master(self.p))

    def info(self):
        v = self.L.nad_pc_info(self.p)
        return {"gpu": bool(v & 1), "oneshot": bool(v & 2), "rccl": bool(v & 4),
                "oneshot_alloc": ("uncached" if v & 8 else "hipMalloc") if v & 2 else None}

    def _err(self, what):
        e = self.L.nad_pc_last_error(self.p)
        return RuntimeError(f"{what} failed: {e.decode() if e else ''}")

    @staticmethod
    def _f32(t):
        import torch
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise TypeError("parallel_context buffers are contiguous float32 tensors")
        return C.c_void_p(t.data_ptr())

    def barrier(self):
        self.L.barrier(self.p)

    def broadcast(self, buffer, root=0):
        """from rank 0 (the reference always broadcasts from the master, parallel_context.cpp:58-61)"""
        if root != 0:
            raise ValueError("broadcast root must be 0 (reference semantics)")
        self.L.broadcast(self.p, self._f32(buffer), buffer.numel())
        return buffer

    def alltoall(self, send, recv):
        """send/recv hold world blocks of send.numel() // world elements each"""
        w = self.get_tp_size()
        self.L.alltoall(self.p, self._f32(send), self._f32(recv), send.numel() // w)
        if send.is_cuda:
            import torch
            torch.cuda.synchronize()
        return recv

    def reduce_add(self, send, recv=None, stream=None):
        """sum over ranks; in place when recv is None.  Device tensors: asynchronous on `stream` (default: torch's
        current stream) -- graph-capturable; host tensors: synchronous (reference reduce_add)."""
        recv = send if recv is None else recv
        if send.is_cuda:
            import torch
            s = stream if stream is not None else torch.cuda.current_stream()
            rc = self.L.nad_pc_allreduce_f32(self.p, self._f32(send), self._f32(recv), send.numel(),
                                             C.c_void_p(s.cuda_stream))
            if rc != 0:
                raise self._err("nad_pc_allreduce_f32")
        else:
            self.L.reduce_add(self.p, self._f32(send), self._f32(recv), send.numel())
        return recv

    def status(self):
        return self.L.nad_pc_status(self.p)

    def max_over_ranks(self, value):
        return float(self.L.nad_pc_max_f64(self.p, float(value)))

    def all_gather_cols(self, local, sizes):
        """concatenate column shards [M, n_r] of every rank into [M, sum n_r] (column-parallel output gather), through
        alltoall: every rank sends its (padded) shard to every rank."""
        import torch
        w = self.get_tp_size()
        m, width = local.shape[0], max(sizes)
        pad = torch.zeros((m, width), dtype=torch.float32, device=local.device)
        pad[:, :local.shape[1]] = local
        send = pad.reshape(1, -1).repeat(w, 1).contiguous()
        recv = torch.empty_like(send)
        self.alltoall(send, recv)
        blocks = recv.reshape(w, m, width)
        return torch.cat([blocks[r, :, :sizes[r]] for r in range(w)], dim=1)

    def destroy(self):
        if self.p:
            self.L.nad_pc_destroy(self.p)
            self.p = None
