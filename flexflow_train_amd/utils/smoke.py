"""One tiny forward + backward of the flagship model (BERT) on cuda:0, used
by __graft_entry__.smoke().  Asserts that the native HIP kernels ran."""
import torch


def run_smoke():
    from flexflow_train_amd import kernels as K
    from flexflow_train_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_train_amd.models.bert import bert_base, build_bert

    assert torch.cuda.is_available(), "smoke() needs a GPU"
    cfg = FFConfig()
    cfg.batch_size = 2
    cfg.print_freq = 0
    m = FFModel(cfg)
    bc = bert_base(num_encoder_layers=2, hidden_size=256, num_heads=4, dim_feedforward=1024, batch_size=2,
                   sequence_length=128)
    build_bert(m, bc)
    m.compile(optimizer=AdamOptimizer(m, alpha=1e-3), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY])
    ex = m.executor
    dev = ex.cfg.device
    feeds = {n: torch.randint(0, 2, ex.local_input_shape(n), device=dev, dtype=torch.int32) for n in ex.inputs}
    feeds["input_ids"] = torch.randint(0, bc.vocab_size, ex.local_input_shape("input_ids"), device=dev,
                                       dtype=torch.int32)
    feeds["position_ids"] = torch.arange(128, device=dev, dtype=torch.int32).expand(2, 128).contiguous()
    labels = torch.randint(0, bc.vocab_size, (2, 128), device=dev)
    before = dict(K.STATS)
    ex.train_step(feeds, labels)
    torch.cuda.synchronize()
    ran = {k: K.STATS[k] - before.get(k, 0) for k in K.STATS}
    for k in ("attention_fwd", "attention_bwd", "layernorm_fwd", "layernorm_bwd", "softmax_ce", "adam_step",
              "embedding_fwd"):
        assert ran.get(k, 0) > 0, f"native kernel {k} did not run"
    pm = ex.perf_metrics()
    assert pm.loss == pm.loss and pm.loss > 0, "bad loss"
    print(f"smoke ok: loss={pm.loss:.4f} kernels={ {k: v for k, v in ran.items() if v} }")
