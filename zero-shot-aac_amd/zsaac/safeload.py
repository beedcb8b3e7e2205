"""Loading the reference's data files without executing code from them.

The reference stores its inputs as pickles: the embedding files written by
data_handing/embeddings_generator.py:64-73 (a list of dicts ``{"audio_embedding": Tensor[1,1024],
"caption": ..., "text_embedding": ..., "audio_id": str}``), ``audioset_label.pkl``
(``{"label_id", "label", "label_embedding": Tensor[1,1024]}`` per label,
dataset/dataset.py:465-474) and the checkpoint ``best.pth`` (a state dict, predict_prompt.py:220).

``load_pickle`` unpickles with an allow-list: containers, strings and numbers, numpy arrays, and
torch tensors.  A pickled torch tensor rebuilds its storage through
``torch.storage._load_from_bytes``, which runs ``torch.load(weights_only=False)`` on the embedded
bytes; that hook is replaced by a ``weights_only=True`` load.  Any other global makes the load
fail with ``pickle.UnpicklingError``.  Checkpoints go through ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import collections
import io
import pickle
from typing import Any, Iterator, List

import numpy as np
import torch


def _storage_from_bytes(b: bytes):
    return torch.load(io.BytesIO(b), weights_only=True)


_ALLOWED = {
    ("builtins", "dict"), ("builtins", "list"), ("builtins", "tuple"), ("builtins", "set"),
    ("builtins", "frozenset"), ("builtins", "str"), ("builtins", "int"), ("builtins", "float"),
    ("builtins", "bool"), ("builtins", "complex"), ("builtins", "bytes"), ("builtins", "bytearray"),
    ("collections", "OrderedDict"),
    ("torch._utils", "_rebuild_tensor_v2"), ("torch._utils", "_rebuild_parameter"),
    ("torch._utils", "_rebuild_tensor"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str) -> Any:
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _storage_from_bytes
        if (module, name) == ("collections", "OrderedDict"):
            return collections.OrderedDict
        if module == "torch" and name.endswith("Storage"):
            return getattr(torch, name)
        if (module, name) in _ALLOWED:
            if module == "builtins":
                import builtins
                return getattr(builtins, name)
            if module == "torch._utils":
                import torch._utils as tu
                return getattr(tu, name)
            if module in ("numpy.core.multiarray", "numpy._core.multiarray"):
                try:
                    from numpy._core import multiarray
                except ImportError:          # numpy < 2
                    from numpy.core import multiarray
                return getattr(multiarray, name)
            return getattr(np, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a data file")


def load_pickle(path: str) -> Any:
    """One object from a pickle file, through the allow-list unpickler."""
    with open(path, "rb") as f:
        return _SafeUnpickler(f).load()


def iter_pickles(path: str) -> Iterator[Any]:
    """Every object of a file holding several consecutive pickles (the reference's text-memory
    files, predict_prompt.py:36-48), through the allow-list unpickler."""
    with open(path, "rb") as f:
        while True:
            try:
                yield _SafeUnpickler(f).load()
            except EOFError:
                return


def load_state_dict(path: str) -> dict:
    """A checkpoint state dict (``best.pth``): tensors only, nothing executed."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]          # the CLAP checkpoints wrap the state dict (predict_prompt.py:126)
    return sd


def as_tensor(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.detach().float().cpu()
    return torch.as_tensor(np.asarray(x), dtype=torch.float32)


def stack_rows(items: List[Any]) -> torch.Tensor:
    return torch.cat([as_tensor(x).reshape(1, -1) for x in items], dim=0)
