"""Text preprocessing (reference: python/flexflow/keras/preprocessing/text.py,
which re-exports keras_preprocessing; implemented here)."""
from __future__ import annotations

import hashlib
import json
from collections import OrderedDict, defaultdict

import numpy as np

_FILTERS = '!"#$%&()*+,-./:;<=>?@[\\]^_`{|}~\t\n'


def text_to_word_sequence(text, filters=_FILTERS, lower=True, split=" "):
    if lower:
        text = text.lower()
    text = text.translate(str.maketrans({c: split for c in filters}))
    return [w for w in text.split(split) if w]


def hashing_trick(text, n, hash_function=None, filters=_FILTERS, lower=True, split=" "):
    if hash_function in (None, "md5"):
        def hash_function(w):
            return int(hashlib.md5(w.encode()).hexdigest(), 16)
    return [hash_function(w) % (n - 1) + 1 for w in text_to_word_sequence(text, filters, lower, split)]


def one_hot(text, n, filters=_FILTERS, lower=True, split=" "):
    return hashing_trick(text, n, hash, filters, lower, split)


class Tokenizer:
    """Word-index tokenizer: fit on texts (or sequences), then map texts to
    index sequences or sequences to (N, num_words) matrices."""

    def __init__(self, num_words=None, filters=_FILTERS, lower=True, split=" ", char_level=False, oov_token=None,
                 document_count=0, **kw):
        self.num_words, self.filters, self.lower, self.split = num_words, filters, lower, split
        self.char_level, self.oov_token = char_level, oov_token
        self.document_count = document_count
        self.word_counts = OrderedDict()
        self.word_docs = defaultdict(int)
        self.index_docs = defaultdict(int)
        self.word_index, self.index_word = {}, {}

    def _words(self, text):
        if self.char_level or isinstance(text, list):
            return [t.lower() for t in text] if self.lower and not isinstance(text, list) else list(text)
        return text_to_word_sequence(text, self.filters, self.lower, self.split)

    def fit_on_texts(self, texts):
        for text in texts:
            self.document_count += 1
            seq = self._words(text)
            for w in seq:
                self.word_counts[w] = self.word_counts.get(w, 0) + 1
            for w in set(seq):
                self.word_docs[w] += 1
        order = sorted(self.word_counts.items(), key=lambda kv: -kv[1])
        vocab = ([self.oov_token] if self.oov_token is not None else []) + [w for w, _ in order]
        self.word_index = {w: i + 1 for i, w in enumerate(vocab)}
        self.index_word = {i: w for w, i in self.word_index.items()}
        for w, c in self.word_docs.items():
            self.index_docs[self.word_index[w]] = c

    def fit_on_sequences(self, sequences):
        self.document_count += len(sequences)
        for seq in sequences:
            for i in set(seq):
                self.index_docs[i] += 1

    def texts_to_sequences(self, texts):
        out = []
        oov = self.word_index.get(self.oov_token) if self.oov_token is not None else None
        for text in texts:
            seq = []
            for w in self._words(text):
                i = self.word_index.get(w)
                if i is not None and (not self.num_words or i < self.num_words):
                    seq.append(i)
                elif oov is not None:
                    seq.append(oov)
            out.append(seq)
        return out

    def sequences_to_texts(self, sequences):
        return [" ".join(self.index_word[i] for i in seq if i in self.index_word) for seq in sequences]

    def sequences_to_matrix(self, sequences, mode="binary"):
        """(N, num_words) matrix; mode binary | count | freq | tfidf."""
        n = self.num_words or (len(self.word_index) + 1)
        if not n:
            raise ValueError("Tokenizer: specify num_words or fit first")
        if mode == "tfidf" and not self.document_count:
            raise ValueError("tfidf needs fit_on_texts / fit_on_sequences first")
        x = np.zeros((len(sequences), n))
        for i, seq in enumerate(sequences):
            counts = defaultdict(int)
            for j in seq:
                if j < n:
                    counts[int(j)] += 1
            for j, c in counts.items():
                if mode == "count":
                    x[i, j] = c
                elif mode == "freq":
                    x[i, j] = c / len(seq)
                elif mode == "binary":
                    x[i, j] = 1
                elif mode == "tfidf":
                    tf = 1 + np.log(c)
                    idf = np.log(1 + self.document_count / (1 + self.index_docs.get(j, 0)))
                    x[i, j] = tf * idf
                else:
                    raise ValueError(f"unknown mode {mode!r}")
        return x

    def texts_to_matrix(self, texts, mode="binary"):
        return self.sequences_to_matrix(self.texts_to_sequences(texts), mode)

    def get_config(self):
        return {"num_words": self.num_words, "filters": self.filters, "lower": self.lower, "split": self.split,
                "char_level": self.char_level, "oov_token": self.oov_token,
                "document_count": self.document_count, "word_counts": json.dumps(self.word_counts),
                "word_index": json.dumps(self.word_index)}

    def to_json(self, **kw):
        return json.dumps({"class_name": "Tokenizer", "config": self.get_config()}, **kw)


def tokenizer_from_json(json_string):
    cfg = json.loads(json_string)["config"]
    wc = json.loads(cfg.pop("word_counts"))
    wi = json.loads(cfg.pop("word_index"))
    t = Tokenizer(**cfg)
    t.word_counts = OrderedDict(wc)
    t.word_index = {k: int(v) for k, v in wi.items()}
    t.index_word = {v: k for k, v in t.word_index.items()}
    return t
