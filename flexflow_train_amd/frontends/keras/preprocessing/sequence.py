"""Sequence preprocessing (reference: python/flexflow/keras/preprocessing/
sequence.py, which re-exports keras_preprocessing; implemented here)."""
from __future__ import annotations

import numpy as np


def pad_sequences(sequences, maxlen=None, dtype="int32", padding="pre", truncating="pre", value=0.0):
    """List of sequences -> (N, maxlen) array, padded / truncated at the
    front ("pre") or back ("post")."""
    seqs = [list(s) for s in sequences]
    maxlen = maxlen if maxlen is not None else max((len(s) for s in seqs), default=0)
    out = np.full((len(seqs), maxlen), value, dtype=dtype)
    for i, s in enumerate(seqs):
        if not s:
            continue
        s = s[-maxlen:] if truncating == "pre" else s[:maxlen]
        if padding == "post":
            out[i, :len(s)] = s
        else:
            out[i, maxlen - len(s):] = s
    return out


def make_sampling_table(size, sampling_factor=1e-5):
    """Zipf-based word sampling probabilities (word2vec subsampling)."""
    gamma = 0.577
    rank = np.arange(size)
    rank[0] = 1
    inv_fq = rank * (np.log(rank) + gamma) + 0.5 - 1.0 / (12.0 * rank)
    f = sampling_factor * inv_fq
    return np.minimum(1.0, f / np.sqrt(f))


def skipgrams(sequence, vocabulary_size, window_size=4, negative_samples=1.0, shuffle=True, categorical=False,
              sampling_table=None, seed=None):
    rng = np.random.default_rng(seed)
    couples, labels = [], []
    for i, wi in enumerate(sequence):
        if not wi:
            continue
        if sampling_table is not None and sampling_table[wi] < rng.random():
            continue
        for j in range(max(0, i - window_size), min(len(sequence), i + window_size + 1)):
            if j != i and sequence[j]:
                couples.append([wi, sequence[j]])
                labels.append([0, 1] if categorical else 1)
    if negative_samples > 0 and couples:
        n = int(len(couples) * negative_samples)
        words = [c[0] for c in couples]
        for _ in range(n):
            couples.append([words[int(rng.integers(len(words)))], int(rng.integers(1, vocabulary_size))])
            labels.append([1, 0] if categorical else 0)
    if shuffle:
        p = rng.permutation(len(couples))
        couples, labels = [couples[k] for k in p], [labels[k] for k in p]
    return couples, labels


def _remove_long_seq(maxlen, seq, label):
    keep = [(s, l) for s, l in zip(seq, label) if len(s) < maxlen]
    return [s for s, _ in keep], [l for _, l in keep]
