"""Host logic of the resample processor's closed-form null keys (kernels.rope_axis_tables, RopeTables; CPU)."""

import torch

from oracle.cogvideox_oracle import prepare_rotary_positional_embeddings


def _rope(F_, Hh, Ww):
    cos, sin = prepare_rotary_positional_embeddings(Hh * 16, Ww * 16, F_, 64)
    return cos.float().contiguous(), sin.float().contiguous()


def test_rope_axis_tables_factor_the_reference_table():
    """CogVideoX's 3D RoPE (embeddings.py:457-530) is the product of per-axis tables: dims 0-15 by frame, 16-39 by
    row, 40-63 by column; the extracted factors rebuild the table exactly."""
    from videopainter_amd import kernels as K
    for grid in ((3, 5, 16), (13, 30, 45), (1, 2, 3)):
        F_, Hh, Ww = grid
        cos, sin = _rope(*grid)
        ax = K.rope_axis_tables((cos, sin), grid)
        assert ax is not None, grid
        ct, st, cy, sy, cx, sx = ax
        assert ct.shape == (F_, 16) and cy.shape == (Hh, 24) and cx.shape == (Ww, 24)
        for tab, (t_, y_, x_) in ((cos, (ct, cy, cx)), (sin, (st, sy, sx))):
            rebuilt = torch.cat([t_[:, None, None, :].expand(F_, Hh, Ww, 16), y_[None, :, None, :].expand(F_, Hh, Ww, 24),
                                 x_[None, None, :, :].expand(F_, Hh, Ww, 24)], -1).reshape(-1, 64)
            assert torch.equal(rebuilt, tab)


def test_rope_axis_tables_reject_other_tables():
    """A table that is not the separable product (one perturbed entry), a wrong grid, or another dtype: None (the
    processor then keeps the null keys as keys)."""
    from videopainter_amd import kernels as K
    cos, sin = _rope(3, 5, 16)
    bad = cos.clone()
    bad[17, 20] += 1e-3
    assert K.rope_axis_tables((bad, sin), (3, 5, 16)) is None
    assert K.rope_axis_tables((cos, sin), (3, 16, 5)) is None
    assert K.rope_axis_tables((cos, sin), (2, 5, 16)) is None
    assert K.rope_axis_tables((cos.double(), sin.double()), (3, 5, 16)) is None
    # cached per table while it is alive and unmodified; an in-place edit bumps the version and re-checks
    good = cos.clone()
    assert K.rope_axis_tables((good, sin), (3, 5, 16)) is not None
    good[0, 0] += 1.0
    assert K.rope_axis_tables((good, sin), (3, 5, 16)) is None


def test_rope_tables_carry_the_grid():
    from videopainter_amd.attention_processor import RopeTables, _rope_dev
    cos, sin = _rope(2, 3, 4)
    r = _rope_dev((cos, sin), torch.device("cpu"), grid=(2, 3, 4))
    assert isinstance(r, RopeTables) and r.grid == (2, 3, 4)
    c2, s2 = r
    assert c2 is cos and s2 is sin
    assert _rope_dev(r, torch.device("cpu")).grid == (2, 3, 4)  # kept through the block's own conversion
    assert _rope_dev((cos, sin), torch.device("cpu")).grid is None
