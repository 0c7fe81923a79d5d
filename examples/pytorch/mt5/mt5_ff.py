"""mT5 (Hugging Face MT5ForConditionalGeneration) trained through the
framework (reference: examples/python/pytorch/mt5/mt5_ff.py).

No network here: the model is built from an MT5Config with random weights
(google/mt5-small's shape by default, a tiny one for quick runs) and trained
on synthetic token data of the reference's shape (source / target length
48, labels shifted by one, pad labels -100 ignored by the loss).  The import
goes through PyTorchModel(is_hf_model=True) -> torch.export -> the ATen
lowering (flexflow_train_amd/frontends/torch_export.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from transformers import MT5Config, MT5ForConditionalGeneration  # noqa: E402

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402
from flexflow.torch.model import PyTorchModel, copy_weights  # noqa: E402


def mt5_config(quick: bool) -> MT5Config:
    if quick:
        return MT5Config(vocab_size=1024, d_model=64, d_kv=16, d_ff=128, num_layers=2, num_decoder_layers=2,
                         num_heads=4, relative_attention_num_buckets=16, dropout_rate=0.0)
    # google/mt5-small
    return MT5Config(vocab_size=250112, d_model=512, d_kv=64, d_ff=1024, num_layers=8, num_decoder_layers=8,
                     num_heads=6, relative_attention_num_buckets=32, dropout_rate=0.0, tie_word_embeddings=False)


def synthetic_data(n, src_len, tgt_len, vocab, seed=42):
    """Token ids of the reference's preprocessing: y_ids = target[:, :-1],
    lm_labels = target[:, 1:], padding -> -100 in the labels."""
    rng = np.random.default_rng(seed)
    ids = rng.integers(1, vocab, (n, src_len))
    mask = np.ones((n, src_len), np.int64)
    lens = rng.integers(src_len // 2, src_len + 1, n)
    for i, ln in enumerate(lens):
        ids[i, ln:] = 0
        mask[i, ln:] = 0
    tgt = rng.integers(1, vocab, (n, tgt_len + 1))
    y_ids, labels = tgt[:, :-1].copy(), tgt[:, 1:].astype(np.int32)
    tl = rng.integers(tgt_len // 2, tgt_len + 1, n)
    for i, ln in enumerate(tl):
        labels[i, ln:] = -100
    return ids, mask, y_ids, labels


def top_level_task():
    quick = "FF_EXAMPLE_SAMPLES" in os.environ
    ffconfig = FFConfig()
    ffconfig.parse_args()
    torch.manual_seed(42)
    model = MT5ForConditionalGeneration(mt5_config(quick))
    n = int(os.environ.get("FF_EXAMPLE_SAMPLES", 1024))
    seq = 16 if quick else 48
    ids, mask, y_ids, labels = synthetic_data(n, seq, seq, model.config.vocab_size)
    bs = ffconfig.batch_size
    ffmodel = FFModel(ffconfig)
    input_tensors = [ffmodel.create_tensor([bs, ids.shape[1]], DataType.DT_INT64, create_grad=False),
                     ffmodel.create_tensor([bs, mask.shape[1]], DataType.DT_INT64, create_grad=False),
                     ffmodel.create_tensor([bs, y_ids.shape[1]], DataType.DT_INT64, create_grad=False)]
    print("Tracing the model...")
    hf_model = PyTorchModel(model, is_hf_model=True, input_names=["input_ids", "attention_mask", "decoder_input_ids"],
                            batch_size=bs, seq_length=(ids.shape[1], y_ids.shape[1]))
    hf_model.torch_to_ff(ffmodel, input_tensors)
    print("Compiling the model...")
    ffmodel.compile(optimizer=SGDOptimizer(ffmodel, lr=0.01), loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    copy_weights(ffmodel)
    print("Creating data loaders...")
    dls = [ffmodel.create_data_loader(t, a) for t, a in zip(input_tensors, (ids, mask, y_ids))]
    labels_dl = ffmodel.create_data_loader(ffmodel.label_tensor, labels)
    ffmodel.init_layers()
    print("Training...")
    ffmodel.fit(x=dls, y=labels_dl, batch_size=bs, epochs=ffconfig.epochs)


if __name__ == "__main__":
    top_level_task()
