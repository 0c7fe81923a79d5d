"""Reuters newswire topics (reference: python/flexflow/keras/datasets/
reuters.py): x is an object array of word-index lists, y int64 topic ids
(46 topics).  Synthetic stand-in: each topic draws most of its words from its
own band of the vocabulary."""
from __future__ import annotations

import numpy as np

from ._synthetic import local_npz

N_TOPICS, N_SAMPLES, VOCAB = 46, 11228, 30979


def load_data(path="reuters.npz", num_words=None, skip_top=0, maxlen=None, test_split=0.2, seed=113, start_char=1,
              oov_char=2, index_from=3, **kw):
    got = local_npz(path)
    if got is not None:
        return got
    rng = np.random.default_rng(seed)
    vocab = VOCAB if not num_words else int(num_words)
    lo = index_from + 1
    band = max(1, (vocab - lo) // N_TOPICS)
    ys = rng.integers(0, N_TOPICS, N_SAMPLES)
    xs = []
    for y in ys:
        n = int(rng.integers(20, 200))
        own = lo + y * band + rng.integers(0, band, n)
        common = rng.integers(lo, vocab, n)
        words = np.where(rng.random(n) < 0.6, own, common)
        words = [int(w) if skip_top <= w < vocab else oov_char for w in words]
        if maxlen:
            words = words[:maxlen - 1]
        xs.append([start_char] + words)
    arr = np.empty(len(xs), dtype=object)
    arr[:] = xs
    cut = int(len(xs) * (1 - test_split))
    return (arr[:cut], ys[:cut].astype(np.int64)), (arr[cut:], ys[cut:].astype(np.int64))


def get_word_index(path="reuters_word_index.json"):
    return {f"word{i}": i for i in range(1, VOCAB)}
