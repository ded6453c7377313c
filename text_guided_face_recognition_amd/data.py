"""Data formats of the reference's text side.

* ``load_caption_store`` reads ``captions_<bert_type>.pickle`` as written by
  utils/dataset_utils.py:183-217: a protocol-2 pickle of
  ``[train_caps, train_masks, valid_caps, valid_masks, test_caps, test_masks]``,
  each a list of per-caption ``LongTensor[L]`` (token ids / attention mask).
* ``load_name_list`` reads the filename / class-id pickles (plain lists).

Both use a restricted unpickler: only the globals a pickled list of CPU
tensors needs are resolved (tensor rebuild, a storage blob loaded with
``torch.load(weights_only=True)``, OrderedDict, the protocol-2 bytes codec);
anything else raises, so a caption file cannot execute code.

``caption_batch`` stacks a batch of captions into the ``[B, L]`` id / mask
tensors the text encoder takes.  Note the reference's training loader bug
(utils/train_dataset.py:81: ``captions[sent_ix]`` instead of
``captions[new_sent_ix]``, so every image draws one of the first captions);
``caption_batch`` indexes what it is given and does not replicate it.
"""
from __future__ import annotations

import codecs
import collections
import io
import pickle

import torch

__all__ = ["load_caption_store", "load_name_list", "caption_batch", "CaptionStore"]


def _storage_from_bytes(b):
    return torch.load(io.BytesIO(b), weights_only=True)


_ALLOWED = {
    ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
    ("torch.storage", "_load_from_bytes"): _storage_from_bytes,
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("_codecs", "encode"): codecs.encode,
}


class _Restricted(pickle.Unpickler):
    def find_class(self, module, name):
        fn = _ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError(f"refusing to load global {module}.{name}")
        return fn


def _load(path):
    with open(path, "rb") as f:
        return _Restricted(f).load()


CaptionStore = collections.namedtuple(
    "CaptionStore", "train_caps train_masks valid_caps valid_masks test_caps test_masks")


def load_caption_store(path):
    """The six caption / mask lists of a ``captions_<bert_type>.pickle``."""
    x = _load(path)
    if not isinstance(x, (list, tuple)) or len(x) != 6:
        raise ValueError(f"{path}: expected the 6-list written by load_text_data_Bert")
    return CaptionStore(*x)


def load_name_list(path):
    """A filename or class-id pickle (a plain list)."""
    x = _load(path)
    if not isinstance(x, (list, tuple)):
        raise ValueError(f"{path}: expected a list")
    return list(x)


def caption_batch(captions, masks, index, device=None):
    """Stack captions[index] / masks[index] into [B, L] LongTensors (all
    captions of one store share L = bert_words_num)."""
    ids = torch.stack([torch.as_tensor(captions[i]).long() for i in index])
    att = torch.stack([torch.as_tensor(masks[i]).long() for i in index])
    if device is not None:
        ids, att = ids.to(device, non_blocking=True), att.to(device, non_blocking=True)
    return ids, att
