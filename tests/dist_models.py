"""Small models used by the multi-process strategy-equivalence tests.
Each function builds the model into an FFModel and returns (feeds, labels)
as GLOBAL tensors (every rank slices its own piece)."""
import torch

from flexflow_train_amd.core import ActiMode, AggrMode, DataType


def mlp(m):
    x = m.create_tensor([16, 32], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 64, ActiMode.AC_MODE_RELU, name="fc0")
    t = m.dense(t, 48, name="fc1")
    t = m.relu(t, name="act1")
    t = m.dense(t, 8, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(7)
    return {"x": torch.randn(16, 32, generator=g)}, torch.randint(0, 8, (16,), generator=g)


def mlp_l2(m):
    """MLP whose first Dense carries an L2 kernel regularizer."""
    x = m.create_tensor([16, 32], DataType.DT_FLOAT, name="x")
    t = m.dense(x, 64, ActiMode.AC_MODE_RELU, kernel_regularizer=("l2", 0.5), name="fc0")
    t = m.dense(t, 48, kernel_regularizer=("l1", 0.05), name="fc1")
    t = m.dense(t, 8, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(9)
    return {"x": torch.randn(16, 32, generator=g)}, torch.randint(0, 8, (16,), generator=g)


def attention(m):
    B, S, E = 4, 8, 32
    x = m.create_tensor([B, S, E], DataType.DT_FLOAT, name="x")
    a = m.multihead_attention(x, x, x, E, 4, name="mha")
    t = m.add(a, x, name="res")
    t = m.layer_norm(t, [-1], name="ln")
    t = m.dense(t, 10, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(11)
    return {"x": torch.randn(B, S, E, generator=g)}, torch.randint(0, 10, (B, S), generator=g)


def embedding(m):
    B, S, V, E = 4, 6, 50, 16
    ids = m.create_tensor([B, S], DataType.DT_INT32, create_grad=False, name="ids")
    t = m.embedding(ids, V, E, AggrMode.AGGR_MODE_NONE, name="emb")
    t = m.dense(t, 12, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(5)
    return ({"ids": torch.randint(0, V, (B, S), generator=g, dtype=torch.int32)},
            torch.randint(0, 12, (B, S), generator=g))


def bert_tiny(m):
    from flexflow_train_amd.models.bert import BertConfig, build_bert

    cfg = BertConfig(vocab_size=64, hidden_size=32, num_heads=4, dim_feedforward=64, num_encoder_layers=2,
                     sequence_length=8, batch_size=4, max_position_embeddings=8, type_vocab_size=2)
    build_bert(m, cfg)
    g = torch.Generator().manual_seed(3)
    B, S = 4, 8
    feeds = {"input_ids": torch.randint(0, 64, (B, S), generator=g, dtype=torch.int32),
             "position_ids": torch.arange(S, dtype=torch.int32).expand(B, S).contiguous(),
             "token_type_ids": torch.randint(0, 2, (B, S), generator=g, dtype=torch.int32)}
    return feeds, torch.randint(0, 64, (B, S), generator=g)


def _seq_attention(m, mode, causal, heads=4):
    B, S, E = 2, 8, 32
    x = m.create_tensor([B, S, E], DataType.DT_FLOAT, name="x")
    a = m.multihead_attention(x, x, x, E, heads, causal=causal, seq_parallel_mode=mode, name="mha")
    t = m.add(a, x, name="res")
    t = m.dense(t, 10, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(13)
    return {"x": torch.randn(B, S, E, generator=g)}, torch.randint(0, 10, (B, S), generator=g)


def attention_ulysses(m):
    return _seq_attention(m, "ulysses", False)


def attention_ring(m):
    return _seq_attention(m, "ring", False)


def attention_ring_causal(m):
    return _seq_attention(m, "ring", True)


def attention_ring_contiguous_causal(m):
    return _seq_attention(m, "ring_contiguous", True)


def attention_ulysses_causal(m):
    return _seq_attention(m, "ulysses", True)


def _moe(m, mode):
    B, D, E, k = 8, 12, 4, 2
    x = m.create_tensor([B, D], DataType.DT_FLOAT, name="x")
    h = m.moe(x, E, k, 16, out_dim=6, expert_parallel_mode=mode, name="moe")
    m.softmax(h, name="sm")
    g = torch.Generator().manual_seed(17)
    return {"x": torch.randn(B, D, generator=g)}, torch.randint(0, 6, (B,), generator=g)


def moe_replicated(m):
    return _moe(m, "replicated")


def moe_alltoall(m):
    return _moe(m, "alltoall")


def cnn(m):
    """conv -> pool -> conv(+residual add) -> relu -> flat -> dense (no BatchNorm:
    per-replica batch statistics make BN intentionally rank-local)."""
    from flexflow_train_amd.core import PoolType
    x = m.create_tensor([8, 3, 12, 12], DataType.DT_FLOAT, name="img")
    t = m.conv2d(x, 8, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_MAX, name="p1")
    u = m.conv2d(t, 8, 3, 3, 1, 1, 1, 1, name="c2")
    t = m.relu(m.add(t, u, name="res"), name="r2")
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_AVG, name="p2")
    t = m.dense(m.flat(t, name="flat"), 6, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(11)
    return {"img": torch.randn(8, 3, 12, 12, generator=g)}, torch.randint(0, 6, (8,), generator=g)


def dlrm_small(m):
    """DLRM-shaped: 4 SUM-bag tables + bottom MLP -> concat -> top MLP ->
    softmax; table layers named like the reference's strategy records
    expect them by index ("embedding<i>" = the i-th embedding)."""
    B, T, V, E = 8, 4, 40, 8
    ids = [m.create_tensor([B, 2], DataType.DT_INT32, create_grad=False, name=f"sparse{i}") for i in range(T)]
    d = m.create_tensor([B, 6], DataType.DT_FLOAT, name="dense")
    x = m.dense(d, E, ActiMode.AC_MODE_RELU, name="bot0")
    embs = [m.embedding(ids[i], V, E, AggrMode.AGGR_MODE_SUM, name=f"emb{i}") for i in range(T)]
    z = m.concat([x] + embs, -1, name="interact")
    t = m.dense(z, 16, ActiMode.AC_MODE_RELU, name="top0")
    t = m.dense(t, 4, name="top1")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(23)
    feeds = {f"sparse{i}": torch.randint(0, V, (B, 2), generator=g, dtype=torch.int32) for i in range(T)}
    feeds["dense"] = torch.randn(B, 6, generator=g)
    return feeds, torch.randint(0, 4, (B,), generator=g)


def towers(m):
    """Two independent Linear towers over one input, summed (inter-operator
    placement: each tower may run on its own devices)."""
    x = m.create_tensor([8, 16], DataType.DT_FLOAT, name="x")
    a = m.dense(x, 32, ActiMode.AC_MODE_RELU, name="a0")
    a = m.dense(a, 12, name="a1")
    b = m.dense(x, 32, ActiMode.AC_MODE_RELU, name="b0")
    b = m.dense(b, 12, name="b1")
    t = m.add(a, b, name="sum")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(3)
    return {"x": torch.randn(8, 16, generator=g)}, torch.randint(0, 12, (8,), generator=g)


def cnn_spatial(m):
    """conv / max pool (padded, stride 2) / conv + residual / padded average
    pool on 16-row images: every window op takes halos from its neighbour
    band when H is sharded (attribute parallelism)."""
    from flexflow_train_amd.core import PoolType
    x = m.create_tensor([4, 3, 16, 10], DataType.DT_FLOAT, name="img")
    t = m.conv2d(x, 8, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    t = m.pool2d(t, 3, 3, 2, 2, 1, 1, PoolType.POOL_MAX, name="p1")
    u = m.conv2d(t, 8, 5, 3, 1, 1, 2, 1, name="c2")
    t = m.relu(m.add(t, u, name="res"), name="r2")
    t = m.pool2d(t, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG, name="p2")
    t = m.dense(m.flat(t, name="flat"), 6, name="out")
    m.softmax(t, name="sm")
    g = torch.Generator().manual_seed(19)
    return {"img": torch.randn(4, 3, 16, 10, generator=g)}, torch.randint(0, 6, (4,), generator=g)
