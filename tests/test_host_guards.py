"""Host-side guards of the kernel wrappers that need no GPU: the pre-split A pieces are
tied to the version of the tensor they were written beside, and caller-supplied outputs are checked
before any launch."""

import pytest
import torch

from robomanipbaselines_amd import kernels as K


def test_presplit_pieces_follow_the_tensor_version():
    y = torch.zeros(4, 8)
    sp = K.PresplitRows(torch.zeros(2, 4, 8, dtype=torch.float16), torch.ones(4))
    assert not sp.valid_for(y)  # never bound
    sp.bind(y)
    y.rmbx_split = sp
    assert K.presplit_of(y) is sp
    assert K.presplit_of(y.view(32)) is None  # a view carries no attribute
    y.add_(1.0)
    assert K.presplit_of(y) is None
    assert K.presplit_of(torch.zeros(4, 8)) is None


def test_groupnorm_act_rejects_a_bad_out_before_launch():
    # host tensors: rejected by the device check before anything is launched
    x = torch.zeros(2, 8, 16)
    w, b = torch.ones(8), torch.zeros(8)
    with pytest.raises(ValueError):
        K.groupnorm_act(x, w, b, 4, out=torch.zeros(2, 8, 16))
