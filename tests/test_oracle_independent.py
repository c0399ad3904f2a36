"""The C oracle against an independent float64 restatement of the reference.

tests/glsl_f64.py states frag.glsl:18-80, vert.glsl:17-22 + rasterisation
coverage and the Vulkan sampler (VulkanCore.cpp:676-710) literally, in float64
numpy, sharing no code, ray basis or padded-texel trick with oracle/vr_oracle.c
(or the HIP library).  Agreement here checks that the oracle -- and so, by the
bit-exact GPU tests, the product -- does not rest on a shared misreading of
the reference.

Bar: on pixels both cover with equal step counts,
|grey difference| <= 1e-5; step-count flips (frag.glsl:46 truncation, fp32
vs fp64) <= 0.01 % of covered pixels; coverage (silhouette) mismatches
<= 0.1 % of pixels.  Measured: max |diff| 8.5e-7 at config
1, <= 7.6e-7 at 1080p x 128 over three views; flips 0-2.9e-5; no coverage
mismatch; CameraPosition off the View eye (five positions, one inside the
box) max 2.9e-6.
"""
import numpy as np
import pytest

import glsl_f64

TOL_GREY = 1e-5
TOL_FLIPS = 1e-4
TOL_COVERAGE = 1e-3


def compare(oracle, vol, obj, glob, m, W, H, rows=None):
    g, n = glsl_f64.render(vol, obj, glob, m, W, H, rows=rows)
    ref, _ = oracle.render(vol, obj, glob, m, W, H, oracle.FMT_RGBA32F)
    no = oracle.step_counts(obj, glob, m, W, H)
    if rows is not None:
        ref, no = ref[rows], no[rows]
    ref = ref[..., 0].astype(np.float64)
    cov_mismatch = ((n >= 0) != (no >= 0)).mean()
    both = (n >= 0) & (no >= 0)
    flips = (both & (n != no)).sum() / max(1, both.sum())
    same = both & (n == no)
    dmax = float(np.abs(g[same] - ref[same]).max()) if same.any() else 0.0
    # uncovered pixels: the oracle keeps the clear colour (VulkanRenderPass.cpp:17-24)
    assert (ref[no < 0] == 0.0).all()
    return dmax, flips, cov_mismatch, int(both.sum())


def test_config1_perlin_cube(oracle):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import perlin_cube_volume
    obj, glob = oracle.reference_shader_data(1.0)
    dmax, flips, cov, covered = compare(oracle, perlin_cube_volume(), obj, glob, oracle.march(32), 256, 256)
    assert covered > 20000
    assert dmax <= TOL_GREY and flips <= TOL_FLIPS and cov <= TOL_COVERAGE, (dmax, flips, cov)


@pytest.fixture(scope="module")
def vol128(oracle):
    return oracle.build_volume(128)


@pytest.mark.parametrize("phi,theta", [(0.0, 0.0), (-120.0, 77.0)])
def test_1080p_128_reference_recipe(oracle, vol128, phi, theta):
    """The config-5 camera and march (1920x1080x128) on the 128^3 recipe
    volume, every 8th row."""
    obj, glob = oracle.reference_shader_data(16 / 9, phi, theta)
    dmax, flips, cov, covered = compare(oracle, vol128, obj, glob, oracle.march(128), 1920, 1080,
                                        rows=np.arange(0, 1080, 8))
    assert covered > 50000
    assert dmax <= TOL_GREY and flips <= TOL_FLIPS and cov <= TOL_COVERAGE, (dmax, flips, cov)


def test_media_scroll_mirrored_repeat(oracle, vol128):
    """Live per-tap MediaScroll offsets push the taps outside [0,1]: the
    Vulkan MIRRORED_REPEAT formula against the oracle's."""
    obj, glob = oracle.reference_shader_data(16 / 9)
    vals = [(0.0, 3.7, -2.2, 1.3), (0.0, -0.6, 5.1, -7.9), (0.0, 1.9, 0.4, -1.1)]
    for col, v in enumerate(vals):
        glob[20 + col * 4:20 + col * 4 + 4] = v
    dmax, flips, cov, _ = compare(oracle, vol128, obj, glob, oracle.march(128), 320, 180)
    assert dmax <= TOL_GREY and flips <= TOL_FLIPS and cov <= TOL_COVERAGE, (dmax, flips, cov)


def test_odd_volume_and_constants(oracle):
    rng = np.random.default_rng(7)
    vol = rng.integers(0, 256, size=(23, 50, 37, 4), dtype=np.uint8)
    obj, glob = oracle.reference_shader_data(1.5, 35.0, -20.0)
    m = oracle.march(96)
    m.density, m.scale, m.step_scale = 2.5, 0.35, 3.0
    m.tap_scale[:] = [0.9, 1.1, 0.5, 1.0]
    dmax, flips, cov, _ = compare(oracle, vol, obj, glob, m, 240, 160)
    # random bytes have gradients of up to 255 per texel, ~50x the noise
    # volumes': the fp32 ray-point drift shows up larger (measured 1.0e-5,
    # flips 1.2e-4)
    assert dmax <= 3e-5 and flips <= 5e-4 and cov <= TOL_COVERAGE, (dmax, flips, cov)


def test_moved_box(oracle):
    """box_min/box_max move the march box and the cube mesh together (they
    coincide in the reference, frag.glsl:31-32 and TestMain.cpp:94-103)."""
    obj, glob = oracle.reference_shader_data(1.5, 35.0, -20.0)
    m = oracle.march(128)
    m.box_min[:] = [-1.5, -0.5, -1.0]
    m.box_max[:] = [1.0, 0.7, 1.8]
    dmax, flips, cov, covered = compare(oracle, oracle.build_volume(48), obj, glob, m, 240, 160)
    assert covered > 5000
    assert dmax <= TOL_GREY and flips <= TOL_FLIPS and cov <= TOL_COVERAGE, (dmax, flips, cov)


@pytest.mark.parametrize("cam", [(4.0, 2.0, 2.5), (0.3, -0.2, 0.5), (1.5, 1.5, 1.5), (-4.0, 1.0, 0.0),
                                 (3.0, 3.0, 3.0001)])
def test_camera_position_off_the_view_eye(oracle, cam):
    """CameraPosition != the View eye (frag.glsl:36-38 with vert.glsl:20):
    the fragment's ray leaves CameraPosition through the front-face point the
    View camera rasterises -- outside the box, inside it (tNear < 0, no clamp
    in frag.glsl) and behind the box."""
    vol = oracle.build_volume(48)
    obj, glob = oracle.reference_shader_data(16 / 9, 20.0, 10.0)
    glob[16:19] = cam
    dmax, flips, cov, covered = compare(oracle, vol, obj, glob, oracle.march(128), 320, 180)
    assert covered > 10000
    assert dmax <= TOL_GREY and flips <= 2e-4 and cov <= TOL_COVERAGE, (dmax, flips, cov)


ANGLES = [(0.0, 0.0), (1.6, 0.0), (30.0, 10.0), (45.0, 45.0), (90.0, 0.0), (-120.0, 77.0), (0.0, 180.0),
          (-75.0, -33.0), (213.3, 12.8), (57.6, 0.0)]


@pytest.mark.parametrize("phi,theta", ANGLES)
def test_w2l_is_glm_float_inverse(oracle, phi, theta):
    """Verdict r04 #6: W2L = glm::inverse(osd.Model) in float
    (TestMain.cpp:230), restated by the product's camera producer
    (vr_camera.cpp), the oracle (vr_oracle.c) and, independently, in numpy
    float32 (tests/glm_f32.py): all three bit for bit."""
    import glm_f32
    from volumetricrenderer_amd import renderer as vrr
    obj, glob = oracle.reference_shader_data(16 / 9, phi, theta)
    osd, gsd = vrr.reference_shader_data(16 / 9, phi, theta)
    pobj, pglob = vrr.shader_data_arrays(osd, gsd)
    want = glm_f32.inverse(obj[:16])
    assert np.array_equal(obj, pobj)
    assert np.array_equal(glob[:16].view(np.uint32), want.view(np.uint32)), (glob[:16], want)
    assert np.array_equal(pglob[:16].view(np.uint32), want.view(np.uint32))
    # and it is an inverse: M * W2L = I to float rounding
    M = obj[:16].reshape(4, 4).T.astype(np.float64)
    L = want.reshape(4, 4).T.astype(np.float64)
    assert np.abs(M @ L - np.eye(4)).max() < 1e-6


def test_glm_inverse_of_a_general_matrix():
    """The numpy restatement on a matrix with every cofactor non-zero (a
    translation, a scale and a shear), against a float64 inverse."""
    import glm_f32
    rng = np.random.default_rng(3)
    for _ in range(20):
        A = rng.normal(size=(4, 4)) + 3 * np.eye(4)
        inv = glm_f32.inverse(A.astype(np.float32).T.reshape(-1)).reshape(4, 4).T
        ref = np.linalg.inv(A.astype(np.float32).astype(np.float64))
        assert np.abs(inv - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("phi,theta", [(30.0, 10.0), (45.0, 45.0), (90.0, 0.0), (0.0, 180.0), (-75.0, -33.0),
                                       (213.3, 12.8)])
def test_rotated_model_views(oracle, phi, theta):
    """Rotated models (the held A/D/W/S keys, TestMain.cpp:177-184, :222-224)
    with the glm W2L: the oracle against the float64 restatement, at the c4
    bars (step-count flips from frag.glsl:46's truncation included)."""
    vol = oracle.build_volume(48)
    obj, glob = oracle.reference_shader_data(16 / 9, phi, theta)
    dmax, flips, cov, covered = compare(oracle, vol, obj, glob, oracle.march(128), 320, 180)
    assert covered > 5000
    assert dmax <= TOL_GREY and flips <= TOL_FLIPS and cov <= TOL_COVERAGE, (dmax, flips, cov)
