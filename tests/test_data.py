"""Caption-store / name-list formats (data.py; reference
utils/dataset_utils.py:183-217): round trip of a protocol-2 pickle laid out
as the reference writes it, and refusal of a pickle carrying any other
global."""
import os
import pickle

import pytest
import torch

from text_guided_face_recognition_amd import data as Dt


def test_caption_store_round_trip(tmp_path):
    caps = [torch.tensor([101, 1000 + i, 2000 + i, 102]) for i in range(5)]
    masks = [torch.ones(4, dtype=torch.long) for _ in range(5)]
    path = tmp_path / "captions_bert.pickle"
    with open(path, "wb") as f:
        pickle.dump([caps, masks, caps[:2], masks[:2], caps[2:], masks[2:]], f, protocol=2)
    st = Dt.load_caption_store(path)
    assert len(st.train_caps) == 5 and len(st.test_masks) == 3
    assert torch.equal(st.train_caps[3], caps[3])
    ids, att = Dt.caption_batch(st.train_caps, st.train_masks, [4, 0])
    assert ids.shape == (2, 4) and ids[0, 1] == 1004 and att.sum() == 8
    names = tmp_path / "filenames.pickle"
    with open(names, "wb") as f:
        pickle.dump(["a/1.jpg", "b/2.jpg"], f, protocol=2)
    assert Dt.load_name_list(names) == ["a/1.jpg", "b/2.jpg"]


class _Evil:
    def __reduce__(self):
        return (os.getenv, ("HOME",))


def test_refuses_other_globals(tmp_path):
    path = tmp_path / "evil.pickle"
    with open(path, "wb") as f:
        pickle.dump([_Evil()], f, protocol=2)
    with pytest.raises(pickle.UnpicklingError):
        Dt.load_name_list(path)
