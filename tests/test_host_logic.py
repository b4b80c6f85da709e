"""Host-side logic that needs no GPU: synthetic workloads, the roofline flop model, the
ABI parameter builders."""
import numpy as np

from cwbl import abi, synth


def test_flop_model_matches_survey():
    # F(40,200) = 1 230 400 flop
    assert synth.flops_per_point(40, 200) == 1_230_400
    assert synth.flops_total(40, 3, 600) == 3 * synth.flops_per_point(40, 200)


def test_synthetic_c2_shapes_and_determinism():
    a = synth.make("c2", scale=0.05, nz=4)
    b = synth.make("c2", scale=0.05, nz=4)
    assert a.var.shape == (40, 4, a.ny, a.nx) and a.var.dtype == np.float32
    assert a.alt.shape == (4, a.ny, a.nx)
    assert a.obs_xyz.shape == (a.obs.shape[0], 3) and a.hdxb.shape == (40, a.obs.shape[0])
    np.testing.assert_array_equal(a.var, b.var)
    np.testing.assert_array_equal(a.hdxb, b.hdxb)


def test_sharded_rows_are_slices_of_the_full_grid():
    full = synth.make("c2", scale=0.05, nz=3)
    part = synth.make("c2", scale=0.05, nz=3, rows=(1, 3))
    np.testing.assert_array_equal(part.var, full.var[:, :, 1::3])
    np.testing.assert_array_equal(part.obs, full.obs)


def test_var_params_defaults_follow_module_config():
    vp = abi.var_params(multi_infl=1.6, use_rtpp=1, rtpp_alpha=0.95)
    assert abs(vp.multi_infl - 1.6) < 1e-7 and vp.use_rtpp == 1 and vp.use_rtps == 0
    assert vp.gts[1].use_it == 0 and vp.radar[1].use_it == 0
    tp = abi.type_params(use_it=1, max_lz_pts=300, hclr=12.0, vclr=3.0, err_muti=[0.5] * 5,
                         is_assim=[1, 0, 1])
    assert list(tp.is_assim) == [1, 0, 1, 1, 1]
    assert tp.max_lz_pts == 300
