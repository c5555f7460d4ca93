"""Drop-in module API on CPU (no kernels run): names, shapes, parameter order,
reference-identical init, checkpoint packages, and loud failure without a GPU."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import ctn_oracle as O


def test_state_dict_matches_reference_fixture():
    import conv_tasnet as ct
    g = np.load(os.path.join(GOLDEN, "model_c1.npz"))
    torch.manual_seed(0)
    m = ct.ConvTasNet(64, 20, 64, 128, 3, 2, 2, 2)
    cfg = O.Cfg(64, 20, 64, 128, 3, 2, 2, 2)
    assert [n for n, _ in m.named_parameters()] == [n for n, _ in O.param_shapes(cfg)]
    for n, p in m.named_parameters():
        ref = g["p:" + n]
        assert tuple(p.shape) == ref.shape, n
        # conv_tasnet.py:41-43 under torch.manual_seed(0): bit-identical to the reference
        assert np.array_equal(p.detach().numpy(), ref), n


@pytest.mark.parametrize("norm,causal", [("gLN", False), ("cLN", True), ("BN", False), ("gLN", True)])
def test_param_names_all_variants(norm, causal):
    import conv_tasnet as ct
    cfg = O.Cfg(16, 8, 8, 16, 3, 3, 2, 3, norm, causal)
    m = ct.ConvTasNet(cfg.N, cfg.L, cfg.B, cfg.H, cfg.P, cfg.X, cfg.R, cfg.C, norm_type=norm, causal=causal)
    assert [(n, tuple(p.shape)) for n, p in m.named_parameters()] == O.param_shapes(cfg)
    assert (m.N, m.L, m.B, m.H, m.P, m.X, m.R, m.C, m.norm_type, m.causal, m.mask_nonlinear) == \
        (16, 8, 8, 16, 3, 3, 2, 3, norm, causal, "relu")


def test_reference_package_loads():
    """A checkpoint written by the reference's own ConvTasNet.serialize loads unchanged."""
    import conv_tasnet as ct
    pkg_path = os.path.join(GOLDEN, "package_tiny.pth")
    m = ct.ConvTasNet.load_model(pkg_path)
    pkg = torch.load(pkg_path, map_location="cpu", weights_only=True)
    assert set(pkg) >= {"N", "L", "B", "H", "P", "X", "R", "C", "norm_type", "causal", "mask_nonlinear",
                        "state_dict", "optim_dict", "epoch", "tr_loss", "cv_loss"}
    for k, v in m.state_dict().items():
        assert torch.equal(v, pkg["state_dict"][k])
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    opt.load_state_dict(pkg["optim_dict"])          # positional Adam state matches parameter order


def test_serialize_roundtrip(tmp_path):
    import conv_tasnet as ct
    torch.manual_seed(3)
    m = ct.ConvTasNet(16, 8, 8, 16, 3, 2, 2, 2, norm_type="cLN", causal=True, mask_nonlinear="softmax")
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    pkg = ct.ConvTasNet.serialize(m, opt, 4, tr_loss=torch.ones(3), cv_loss=torch.zeros(3))
    path = tmp_path / "final.pth.tar"
    torch.save(pkg, path)
    m2 = ct.ConvTasNet.load_model(str(path))
    assert (m2.norm_type, m2.causal, m2.mask_nonlinear) == ("cLN", True, "softmax")
    for (k, v), (k2, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)


def test_cpu_tensors_fail_loudly():
    import conv_tasnet as ct
    import ctn_lib as L
    import pit_criterion as pc
    m = ct.ConvTasNet(16, 8, 8, 16, 3, 2, 2, 2)
    with pytest.raises(L.CtnLibraryError, match="ROCm device only"):
        m(torch.randn(1, 64))
    with pytest.raises(L.CtnLibraryError):
        pc.cal_loss(torch.randn(1, 2, 64), torch.randn(1, 2, 64), torch.tensor([64]))


def test_overlap_and_add_utility():
    import utils
    g = np.load(os.path.join(GOLDEN, "ops.npz"))
    np.testing.assert_array_equal(utils.overlap_and_add(torch.from_numpy(g["ola.kat.sig"]), 2).numpy(),
                                  g["ola.kat.out"])
    for L, S in ((20, 10), (16, 8), (15, 7), (6, 3)):
        np.testing.assert_allclose(utils.overlap_and_add(torch.from_numpy(g[f"ola{L}_{S}.sig"]), S).numpy(),
                                   g[f"ola{L}_{S}.out"], rtol=1e-6, atol=1e-6)


def test_remove_pad():
    import utils
    x = torch.arange(24.).view(2, 3, 4)
    out = utils.remove_pad(x, torch.tensor([4, 2]))
    assert out[0].shape == (3, 4) and out[1].shape == (3, 2)
    assert np.array_equal(out[1], x[1, :, :2].numpy())
