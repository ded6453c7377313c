"""The ``args`` bag the reference's losses and trainers read
(cfg/train_bert.yml, merged over argparse by utils/utils.py:32-44)."""
from __future__ import annotations

import yaml


class AttrDict(dict):
    """EasyDict-style attribute access (the reference uses easydict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    @classmethod
    def wrap(cls, d):
        if isinstance(d, dict):
            return cls({k: cls.wrap(v) for k, v in d.items()})
        return d


DEFAULTS = {
    # cfg/train_bert.yml
    "manual_seed": 100, "CUDA": True,
    "is_DAMSM": True, "is_CLIP": True, "is_CMP": False, "is_WRA": False,
    "is_ident_loss": True, "lambda_clip": 2.0, "lambda_id": 100,
    "aux_feat_dim_per_granularity": 256, "img_size": 112, "model_type": "arcface",
    "num_classes": 4500, "init_lr_bert": 7e-5, "min_lr_bert": 2e-5, "lr_head": 0.001,
    "weight_decay": 0.01, "clip_max_norm": 1.0, "batch_size": 64,
    "TRAIN": {"FLAG": True, "SMOOTH": {"GAMMA1": 4.0, "GAMMA2": 5.0, "GAMMA3": 10.0}},
    "en_type": "BERT", "bert_words_num": 32, "captions_per_image": 10,
    # build-specific
    "precision": "fp32",
}


# cfg/train_lstm.yml (stage 1 with the BiLSTM text encoder, BASELINE configs[0])
LSTM_DEFAULTS = {
    "en_type": "LSTM", "lambda_clip": 1.0, "lambda_id": 100, "lr_head": 0.002,
    "weight_decay": 0.0001, "clip_max_norm": 0.5, "batch_size": 128, "init_lr_lstm": 0.001,
    "min_lr_lstm": 0.00009, "lstm_words_num": 18, "embedding_dim": 256,
    "captions_per_image": 4, "num_classes": 4500,
}


def _coerce(v):
    # cfg/train_bert.yml:35 ships "min_lr_bert: 0.00002)" which YAML reads as a
    # string; the reference then fails in Adam(lr=str).  Coerce numeric strings.
    if isinstance(v, str):
        try:
            return float(v.rstrip(")"))
        except ValueError:
            return v
    return v


def make_args(yaml_path=None, lstm=False, **overrides):
    """cfg/train_bert.yml defaults (cfg/train_lstm.yml with lstm=True), then a
    YAML file's keys, then keyword overrides."""
    cfg = dict(DEFAULTS)
    if lstm:
        cfg.update(LSTM_DEFAULTS)
    if yaml_path:
        with open(yaml_path) as f:
            loaded = yaml.safe_load(f) or {}
        cfg.update({k: _coerce(v) for k, v in loaded.items()})
    cfg.update(overrides)
    args = AttrDict.wrap(cfg)
    return args
