"""Tensor-parallel sharding of packed WOQ weights and the row/column-parallel linears of docs/tensor_parallelism.md.

Split rules follow model_load_tensor::calc_split_type (neural_speed/models/model_utils/model_files.h:134-191):
  TP_1D_ROW    (split ne[1] = N, output features; Megatron "column-parallel"): attention.wq/wk/wv, feed_forward.w1/w3
  TP_1D_COLUMN (split ne[0] = K, input features;  Megatron "row-parallel"):   attention.wo, feed_forward.w2 -> all-reduce
Shards are cut from the packed blob exactly (nad_blob_split: whole 16-wide N stripes / whole quantization groups
along K).  The reference instead dequantizes, slices and re-quantizes (model_files.h:1538-1563), which changes the
weights; here TP=W reproduces TP=1 up to the order of the all-reduce sum.
"""
from . import bestla

TP_1D_ROW = "TP_1D_ROW"
TP_1D_COLUMN = "TP_1D_COLUMN"

_ROW = (".attention.wq.weight", ".attention.wk.weight", ".attention.wv.weight", ".feed_forward.w1.weight",
        ".feed_forward.w3.weight", ".attn.q_proj.weight", ".attn.k_proj.weight", ".attn.v_proj.weight",
        ".mlp.gate_proj.weight", ".mlp.up_proj.weight", ".mlp.fc_in.weight", ".mlp.dense_h_to_4h.weight")
_COL = (".attention.wo.weight", ".feed_forward.w2.weight", ".attn.out_proj.weight", ".self_attn.o_proj.weight",
        ".mlp.down_proj.weight", ".mlp.fc_out.weight", ".self_attention.dense.weight", ".mlp.dense_4h_to_h.weight")


def split_type(name):
    if any(s in name for s in _ROW):
        return TP_1D_ROW
    if any(s in name for s in _COL):
        return TP_1D_COLUMN
    return None


def shard_blob(blob, mode, rank, world, unit=1):
    """(shard blob, (begin, end)) of `rank`: TP_1D_ROW splits N in chunks of `unit` columns -- pass the group size of
    the row-parallel weight that consumes this output (and a multiple of the head size for Q/K/V) so the column
    shards line up with its K shards; TP_1D_COLUMN splits K by whole quantization groups."""
    axis = 0 if mode == TP_1D_ROW else 1
    if world == 1:
        inf = bestla.blob_info(blob)
        return blob, (0, inf["n"] if axis == 0 else inf["k"])
    return bestla.split(blob, axis, rank, world, unit), bestla.split_range(blob, axis, rank, world, unit)


class ColumnParallelLinear:
    """TP_1D_ROW weight: y_local[M, N_r] = x[M, K] . W_r^T (no communication)."""

    def __init__(self, weight, n_range):
        self.weight, self.n_range = weight, n_range

    def __call__(self, x, out=None):
        return self.weight.forward(x, out=out)


class RowParallelLinear:
    """TP_1D_COLUMN weight: y[M, N] = sum_r x[:, K_r] . W_r^T  -> reduce_add (ne_all_reduce, ne_layers.c:1718-1733)."""

    def __init__(self, weight, k_range, ctx):
        self.weight, self.k_range, self.ctx = weight, k_range, ctx

    def __call__(self, x_local, out=None):
        y = self.weight.forward(x_local, out=out)
        if self.ctx is not None and self.ctx.get_tp_size() > 1:
            self.ctx.reduce_add(y)
        return y

    def slice_input(self, x_full):
        lo, hi = self.k_range
        return x_full[:, lo:hi]
