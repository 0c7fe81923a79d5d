"""File cache helper (reference: python/flexflow/keras/utils/data_utils.py).
There is no network here: ``get_file`` returns the cached copy under
``cache_dir`` (default ~/.keras/datasets) and raises when it is absent."""
from __future__ import annotations

import hashlib
import os


def _hash(path, algorithm="sha256", chunk=1 << 20):
    h = hashlib.md5() if algorithm == "md5" else hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(chunk), b""):
            h.update(blk)
    return h.hexdigest()


def validate_file(fpath, file_hash, algorithm="auto"):
    algo = "sha256" if algorithm == "sha256" or (algorithm == "auto" and len(file_hash) == 64) else "md5"
    return _hash(fpath, algo) == str(file_hash)


def get_file(fname, origin=None, untar=False, md5_hash=None, file_hash=None, cache_subdir="datasets",
             hash_algorithm="auto", extract=False, archive_format="auto", cache_dir=None):
    base = cache_dir or os.path.join(os.path.expanduser("~"), ".keras")
    path = os.path.join(base, cache_subdir, fname)
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} is not cached and there is no network access to fetch {origin}")
    want = file_hash or md5_hash
    if want and os.path.isfile(path) and not validate_file(path, want, "md5" if md5_hash else hash_algorithm):
        raise ValueError(f"{path}: hash mismatch")
    return path
