"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

The bar is bit-exact for fp32 output (both sides execute
the same fp32 operation sequence with explicit fma only), bit-exact for
RGBA8 UNORM, and <= 1 LSB for sRGB (powf differs between libm and the device
library).  Executed step counts must match exactly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd import VRError


@pytest.fixture(scope="module")
def r():
    with vr.Renderer(0) as rr:
        yield rr


@pytest.fixture(scope="module")
def vol128(oracle):
    return oracle.build_volume(128)


def render_both(r, oracle, vol, W, H, osd=None, gsd=None, march=None, fmt=0, **band):
    if osd is None:
        osd, gsd = vr.reference_shader_data(W / H)
    march = march if march is not None else vr.march_defaults()
    r.set_volume(vol)
    r.set_shader_data(osd, gsd)
    r.set_march(march)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    img = r.render(W, H, fmt, step_counter=cnt, **band)
    torch.cuda.synchronize()
    obj, glob = vr.shader_data_arrays(osd, gsd)
    ref, steps = oracle.render(vol, obj, glob, oracle.from_params(march), W, H, fmt, **band)
    return img.cpu().numpy(), ref, int(cnt.item()), steps


def assert_exact(img, ref):
    assert img.shape == ref.shape
    bad = np.argwhere(img != ref)
    assert bad.size == 0, f"{len(bad)} mismatches, first {bad[:5].tolist()}: " \
                          f"{img[tuple(bad[0])]} vs {ref[tuple(bad[0])]}"


# layouts measured slower than the auto ones, built only with VR_EXPERIMENTS
# (make EXPERIMENTS=1; vr_internal.h layout_built)
EXPERIMENTAL_LAYOUTS = {2, 3, 4, 6, 7, 8, 9, 10, 11, 13, 16}


def need_experiments(r, what):
    """Skip unless the library was built with the measured-slower variants."""
    if r.get_option("experiments") != 1:
        pytest.skip(f"{what}: built only with VR_EXPERIMENTS (make EXPERIMENTS=1)")


def perlin_cube_volume(oracle, n=128):
    """BASELINE config 1 volume: single-octave Perlin (f=.19, seed 3),
    normalised and inverted as TestMain.cpp:64-78, in all four channels."""
    g, mn, mx = oracle.noise_grid(oracle.NOISE_PERLIN, n, n, n, 0.19, 3)
    inv = np.float32(1.0) / (np.float32(mx) - np.float32(mn))
    s = (np.float32(1.0) - (g - np.float32(mn)) * inv).astype(np.float32)
    b = (s * np.float32(255.0)).astype(np.int32).astype(np.uint8)
    return np.repeat(b[..., None], 4, axis=3)


def test_config1_perlin_cube_256_32(r, oracle):
    vol = perlin_cube_volume(oracle)
    osd, gsd = vr.reference_shader_data(1.0)
    img, ref, c, s = render_both(r, oracle, vol, 256, 256, osd, gsd, vr.march_defaults(max_steps=32))
    assert_exact(img, ref)
    assert c == s == 225872  # 2.26e5
    img8, ref8, _, _ = render_both(r, oracle, vol, 256, 256, osd, gsd, vr.march_defaults(max_steps=32),
                                   fmt=vr.FMT_RGBA8_UNORM)
    assert_exact(img8, ref8)


def test_reference_frame_1080p_128(r, oracle, vol128):
    img, ref, c, s = render_both(r, oracle, vol128, 1920, 1080)
    assert "_clamp" in r.kernel_variant   # the fast clamp path, not planar mirror
    assert_exact(img, ref)
    assert c == s
    assert 16_700_000 < s < 16_780_000  # 1.674e7 executed steps


@pytest.mark.parametrize("phi,theta", [(30.0, 10.0), (45.0, 45.0), (90.0, 0.0), (-120.0, 77.0), (0.0, 180.0)])
def test_rotated_cube(r, oracle, vol128, phi, theta):
    osd, gsd = vr.reference_shader_data(16 / 9, phi, theta)
    img, ref, c, s = render_both(r, oracle, vol128, 320, 180, osd, gsd)
    assert_exact(img, ref)
    assert c == s


SPIN_DEG = 1.6   # TestMain.cpp:171-184, :222-224: 100 deg/s held key x 0.016 s per frame


@pytest.mark.parametrize("layout", [0, 12, 15])
@pytest.mark.parametrize("gpu,interval", [(1, 32), (0, 32), (1, 1), (1, 7)])
def test_spinning_camera_frames(r, oracle, vol128, layout, gpu, interval):
    """A moving camera (verdict r02 #3): 40 consecutive frames, each with new
    shader data (phi += 1.6 deg, the reference's held A/D key).  The region
    lists of the first frame (built on the host: a new target) are reused while
    the camera moves and rebuilt every `interval` renders -- on the GPU
    (vr_regions.hip, option region_gpu 1, the default) or on the host -- so
    frames 1, 33 and 40 cover a reused list, a rebuild and the lists after it;
    each is checked bit-exactly against the oracle, with its step count (a
    tile listed twice would count its steps twice; one left out keeps the
    target's garbage).  Layout 0 = auto (cornerh at 128^3), 12 = brick4832,
    15 = col48 (the config-5 layout)."""
    W, H = 320, 180
    r.set_volume(vol128)
    r.set_layout_preference(layout)
    r.set_march(vr.march_defaults())
    r.set_option("region_gpu", gpu)
    r.set_option("region_interval", interval)
    keep = {1: None, 33: None, 40: None}
    try:
        builds0 = r.get_option("region_gpu_builds")
        for i in range(1, 41):
            osd, gsd = vr.reference_shader_data(W / H, SPIN_DEG * i, 0.0)
            r.set_shader_data(osd, gsd)
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            img = r.alloc_target(W, H, 0)
            img.fill_(float("nan"))
            r.render(W, H, 0, out=img, step_counter=cnt)
            if i in keep:
                keep[i] = (img, cnt, osd, gsd)
        torch.cuda.synchronize()
        builds = r.get_option("region_gpu_builds") - builds0
        if gpu:
            assert builds >= 39 // interval - 1, builds
        else:
            assert builds == 0
        for i, (img, cnt, osd, gsd) in keep.items():
            obj, glob = vr.shader_data_arrays(osd, gsd)
            ref, steps = oracle.render(vol128, obj, glob, oracle.from_params(vr.march_defaults()), W, H, 0)
            assert_exact(img.cpu().numpy(), ref)
            assert int(cnt.item()) == steps, i
    finally:
        r.set_option("region_gpu", 1)
        r.set_option("region_interval", 32)
        r.set_layout_preference(0)


@pytest.mark.parametrize("shadow", [0, 8])
def test_spinning_camera_procedural(r, oracle, shadow):
    """The procedural march under a moving camera: every frame has new
    geometry.  With sort_reuse = 31 the cost sort (bin, scan, scatter) is built
    at frame 1 and again at frame 33; frames in between march the stale order
    of an older camera and, in the trailing blocks, the pixels it left out
    (vr_render SORT_STALE).  Frames 1, 2, 32, 33 and 40 of a 1.6-degree spin
    equal the oracle bit for bit, step counts included; by frame 32 the cube
    has turned ~50 degrees, so many pixels changed coverage.  With sort_reuse
    0 (the default) every frame sorts again."""
    W, H = 160, 96
    m = vr.march_defaults(max_steps=64)
    r.set_march(m)
    r.set_procedural(shadow_steps=shadow)
    p = oracle.procedural_from(r.procedural)
    keep = {}
    try:
        for reuse in ((31, 0) if r.get_option("experiments") == 1 else (0,)):   # sort_reuse: VR_EXPERIMENTS
            r.set_option("sort_reuse", reuse)
            assert r.get_option("sort_reuse") == reuse
            for i in range(1, 41):
                osd, gsd = vr.reference_shader_data(W / H, SPIN_DEG * i, 0.0)
                r.set_shader_data(osd, gsd)
                cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
                img = r.render(W, H, 0, step_counter=cnt)
                if i in (1, 2, 32, 33, 40) and (reuse or i == 2):
                    keep[(reuse, i)] = (img, cnt, osd, gsd)
        torch.cuda.synchronize()
    finally:
        r.set_option("sort_reuse", 0)
        r.set_procedural(enabled=0)
    for (reuse, i), (img, cnt, osd, gsd) in keep.items():
        obj, glob = vr.shader_data_arrays(osd, gsd)
        ref, steps = oracle.render_procedural(p, obj, glob, oracle.from_params(m), W, H, 0)
        assert_exact(img.cpu().numpy(), ref)
        assert int(cnt.item()) == steps, (reuse, i)


def test_media_scroll_mirrored_repeat(r, oracle, vol128):
    osd, gsd = vr.reference_shader_data(16 / 9)
    # per-tap offsets well outside [0,1]: exercises MIRRORED_REPEAT
    for col, vals in enumerate([(0.0, 3.7, -2.2, 1.3), (0.0, -0.6, 5.1, -7.9), (0.0, 1.9, 0.4, -1.1)]):
        for row, v in enumerate(vals):
            gsd.media_scroll[col * 4 + row] = v
    r.set_volume(vol128)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults())
    assert r.kernel_variant == "grid_planar_mirror"
    img, ref, c, s = render_both(r, oracle, vol128, 320, 180, osd, gsd)
    assert_exact(img, ref)


@pytest.mark.parametrize("layout,name", [(1, "planar"), (2, "brick5"), (3, "brick8"), (4, "brick16"), (5, "corner8"),
                                         (6, "brick4"), (7, "zpair"), (8, "brick448"),
                                         (9, "brick488"), (10, "brick4816"), (11, "brick41616"),
                                         (12, "brick4832"), (13, "brick4864"), (14, "cornerh"), (15, "col48"),
                                         (16, "col48z")])
def test_every_layout_bitexact(r, oracle, vol128, layout, name):
    if layout in EXPERIMENTAL_LAYOUTS:
        need_experiments(r, name)
    osd, gsd = vr.reference_shader_data(16 / 9, 20.0, -35.0)
    r.set_volume(vol128)
    r.set_layout_preference(layout)
    try:
        img, ref, c, s = render_both(r, oracle, vol128, 480, 270, osd, gsd)
        # the recipe's constant G (uniform_mask 2) skips its loads in the three regions kernels
        um = r.get_option("uniform_mask")
        suffix = "_uG" if um == 2 and name in ("col48", "brick4832", "cornerh", "col48z") else ""
        assert r.kernel_variant == f"grid_{name}_clamp{suffix}"
        assert_exact(img, ref)
        assert c == s
        # odd, non-power-of-two extents exercise the brick edges
        rng = np.random.default_rng(layout)
        for dims in [(13, 22, 9), (30, 31, 32), (61, 17, 45)]:
            vol = rng.integers(0, 256, size=dims + (4,), dtype=np.uint8)
            img, ref, c, s = render_both(r, oracle, vol, 160, 90, osd, gsd)
            assert_exact(img, ref)
    finally:
        r.set_layout_preference(0)


@pytest.mark.parametrize("layout", [15, 12, 14, 16])
def test_uniform_channel_skip_bitexact(r, oracle, layout):
    """A channel whose texels are all equal (the reference recipe's G,
    TestMain.cpp:60/76) is detected at install (vr_get_option "uniform_mask")
    and its tap becomes the constant v/255 with no load -- exact, because the
    spec's lerps of equal values return them.  Bit-exact with step counts for
    each single uniform channel, with uniform_skip on and off, for the one-lane
    march and the step-split march (split 2 and 4, banded), and for two uniform
    channels (the general kernel)."""
    if layout in EXPERIMENTAL_LAYOUTS:
        need_experiments(r, "col48z")
    rng = np.random.default_rng(layout)
    base = rng.integers(0, 256, size=(40, 44, 36, 4), dtype=np.uint8)
    r.set_layout_preference(layout)
    try:
        for mask in (1, 2, 4, 8, 2 | 8):
            vol = base.copy()
            for ch in range(4):
                if mask >> ch & 1:
                    vol[..., ch] = 17 + 40 * ch
            r.set_volume(vol)
            assert r.get_option("uniform_mask") == mask
            osd, gsd = vr.reference_shader_data(16 / 9, 20.0, -15.0)
            for skip in (1, 0):
                r.set_option("uniform_skip", skip)
                img, ref, c, s = render_both(r, oracle, vol, 320, 180, osd, gsd)
                assert_exact(img, ref)
                assert c == s
                single = mask in (1, 2, 4, 8)
                assert r.kernel_variant.endswith("_u" + "RGBA"[(mask & -mask).bit_length() - 1]) == (skip and single)
            for split in (2, 4):
                r.set_option("split", split)
                img, ref, c, s = render_both(r, oracle, vol, 320, 180, osd, gsd, band_rows=16, band_stride=3,
                                             band_first=1)
                assert_exact(img, ref)
                assert c == s
            r.set_option("split", 0)
    finally:
        r.set_option("uniform_skip", 1)
        r.set_option("split", 0)
        r.set_layout_preference(0)


@pytest.mark.parametrize("dims", [(13, 22, 9), (7, 5, 3), (64, 64, 64)])
def test_uniform_detection_edges(r, dims):
    """k_plane_minmax on planes that start off a 4-byte boundary (odd texel
    counts) and tiny ones: a channel is uniform only if every byte is, so a
    single different byte at the first or the last texel of the plane clears
    its bit."""
    rng = np.random.default_rng(sum(dims))
    for ch in range(4):
        vol = rng.integers(0, 256, size=tuple(reversed(dims)) + (4,), dtype=np.uint8)
        vol[..., ch] = 200
        r.set_volume(vol)
        assert r.get_option("uniform_mask") == 1 << ch
        for idx in ((0, 0, 0), (-1, -1, -1)):
            v2 = vol.copy()
            v2[idx + (ch,)] = 201
            r.set_volume(v2)
            assert r.get_option("uniform_mask") == 0, (ch, idx)


def test_reference_recipe_green_channel_is_uniform(r):
    """The recipe replicates TestMain.cpp:60 (the f=.03 grid written into
    noiseOutput1), so noiseOutput2 stays zero and G is one constant byte
    (SURVEY.md sec. 8 a8): the install finds channel G (bit 1) uniform."""
    r.generate_volume(vr.volume_recipe_defaults(size=48))
    assert r.get_option("uniform_mask") == 2
    r.generate_volume(vr.volume_recipe_defaults(size=48, literal_overwrite=0))
    assert r.get_option("uniform_mask") == 0


@pytest.mark.parametrize("layout", [15, 12, 14])
def test_region_workgroups_and_supertiles_bitexact(r, oracle, vol128, layout):
    """Regions schedule with 8 or 16 waves per workgroup (wg_waves) and the
    list ordered per tile or by 4x4 blocks of tiles (supertile; 2x2 is the
    default every other test runs): only the order and
    the grouping of tiles change, so every frame is bit-exact, step counts
    included; also a banded target and early-out."""
    r.set_volume(vol128)
    r.set_layout_preference(layout)
    try:
        exp = r.get_option("experiments") == 1   # 8 / 16-wave workgroups: VR_EXPERIMENTS only
        for wg, st in [(4, 1), (8, 1), (16, 1), (4, 4), (8, 2), (16, 4)]:
            if wg != 4 and not exp:
                continue
            r.set_option("wg_waves", wg)
            r.set_option("supertile", st)
            assert (r.get_option("wg_waves"), r.get_option("supertile")) == (wg, st)
            for (W, H, phi, theta) in [(480, 270, 0.0, 0.0), (203, 117, 35.0, -20.0)]:
                osd, gsd = vr.reference_shader_data(W / H, phi, theta)
                img, ref, c, s = render_both(r, oracle, vol128, W, H, osd, gsd)
                assert_exact(img, ref)
                assert c == s
        osd, gsd = vr.reference_shader_data(16 / 9, -40.0, 15.0)
        img, ref, c, s = render_both(r, oracle, vol128, 320, 180, osd, gsd, march=vr.march_defaults(early_out=0.5),
                                     band_rows=16, band_stride=3, band_first=1)
        assert_exact(img, ref)
        assert c == s
    finally:
        r.set_option("wg_waves", 4)
        r.set_option("supertile", 2)
        r.set_layout_preference(0)


@pytest.mark.parametrize("cap", [32, 12, 0])
def test_slab_march_bitexact(r, oracle, vol128, cap):
    """The LDS-slab march (COL48 + option slab, vr_march_slab.hip): per step a
    wave fills its box of 64-B chunks per channel into LDS and reads its taps
    there; a channel whose box exceeds slab_cap chunks reads straight from the
    layout.  cap 32 = the full slab, 12 = a mix of slab and fallback channels,
    0 = every channel falls back.  Bit-exact vs the oracle with step counts:
    the reference view and rotated views at 128^3, odd extents, a 200^3
    random volume on a small frame (big boxes), early-out, MediaScroll offsets
    inside the clamp-exact range (the non-zero-offset kernel).  The slab
    march is in the default library (option slab, off by default)."""
    r.set_volume(vol128)
    r.set_layout_preference(15)
    r.set_option("slab", 1)
    r.set_option("slab_cap", cap)
    try:
        for (W, H, phi, theta) in [(480, 270, 0.0, 0.0), (320, 180, 20.0, -35.0), (200, 120, -75.0, 60.0)]:
            osd, gsd = vr.reference_shader_data(W / H, phi, theta)
            img, ref, c, s = render_both(r, oracle, vol128, W, H, osd, gsd)
            assert r.kernel_variant == "grid_col48_slab_clamp"
            assert_exact(img, ref)
            assert c == s
        rng = np.random.default_rng(cap + 5)
        osd, gsd = vr.reference_shader_data(16 / 9, 10.0, 25.0)
        for dims in [(13, 22, 9), (61, 17, 45), (200, 200, 200)]:
            vol = rng.integers(0, 256, size=dims + (4,), dtype=np.uint8)
            img, ref, c, s = render_both(r, oracle, vol, 96, 54, osd, gsd)
            assert_exact(img, ref)
            assert c == s
        # early-out, and small per-tap offsets (stays clamp-exact: the plain T path)
        vol = rng.integers(0, 256, size=(40, 40, 40, 4), dtype=np.uint8)
        osd, gsd = vr.reference_shader_data(16 / 9, 30.0, 5.0)
        gsd.media_scroll[1 * 4 + 1] = 0.01
        gsd.media_scroll[2 * 4 + 2] = -0.02
        m = vr.march_defaults(early_out=0.6)
        img, ref, c, s = render_both(r, oracle, vol, 160, 90, osd, gsd, march=m)
        assert r.kernel_variant == "grid_col48_slab_clamp_early"
        assert_exact(img, ref)
        assert c == s
    finally:
        r.set_option("slab", 0)
        r.set_option("slab_cap", 32)
        r.set_layout_preference(0)


@pytest.mark.parametrize("schedule,wps", [(0, 4), (1, 1), (1, 3), (1, 8), (2, 1), (2, 3), (2, 16), (3, 1), (4, 1), (4, 2),
                                          (4, 5), (5, 1), (5, 2), (5, 7)])
def test_schedules_bitexact(r, oracle, vol128, schedule, wps):
    if schedule in (1, 2, 3):   # queue, strided, XCD rows: measured slower
        need_experiments(r, f"schedule {schedule}")
    sched0, tpw0 = r.get_option("schedule"), r.get_option("tiles_per_wave")
    r.set_option("schedule", schedule)
    r.set_option("waves_per_simd" if schedule == 1 else "tiles_per_wave", wps)
    try:
        for W, H, band in [(333, 187, {}), (640, 360, dict(band_rows=16, band_stride=3, band_first=2))]:
            img, ref, c, s = render_both(r, oracle, vol128, W, H, **band)
            assert_exact(img, ref)
            assert c == s
    finally:
        r.set_option("schedule", sched0)
        r.set_option("tiles_per_wave", tpw0)
        r.set_option("waves_per_simd", 4)


@pytest.mark.parametrize("dims", [(37, 50, 23), (1, 1, 1), (2, 3, 5), (129, 64, 96)])
def test_odd_volume_dims(r, oracle, dims):
    rng = np.random.default_rng(sum(dims))
    nx, ny, nz = dims
    vol = rng.integers(0, 256, size=(nz, ny, nx, 4), dtype=np.uint8)
    img, ref, c, s = render_both(r, oracle, vol, 200, 120)
    assert_exact(img, ref)
    assert c == s


@pytest.mark.parametrize("steps", [1, 7, 100, 256, 300])
def test_max_steps(r, oracle, vol128, steps):
    img, ref, c, s = render_both(r, oracle, vol128, 256, 144, march=vr.march_defaults(max_steps=steps))
    assert_exact(img, ref)
    assert c == s


def test_box_and_constants(r, oracle, vol128):
    m = vr.march_defaults(box_min=[-1.5, -0.5, -1.0], box_max=[1.0, 0.7, 1.8], density=2.5, scale=0.35,
                          step_scale=3.0, tap_scale=[0.9, 1.1, 0.5, 1.0])
    img, ref, c, s = render_both(r, oracle, vol128, 300, 200, march=m)
    assert_exact(img, ref)
    assert c == s


def test_early_out(r, oracle, vol128):
    m = vr.march_defaults(density=400.0, early_out=0.05)
    img, ref, c, s = render_both(r, oracle, vol128, 320, 180, march=m)
    assert r.kernel_variant.endswith("_early")
    assert_exact(img, ref)
    assert c == s
    m0 = vr.march_defaults(density=400.0)
    full, _, c0, _ = render_both(r, oracle, vol128, 320, 180, march=m0)
    assert c < c0                                     # the early-out fired
    assert np.abs(full - img).max() <= 0.05 + 1e-6    # and cost < eps


def test_formats(r, oracle, vol128):
    img, ref, _, _ = render_both(r, oracle, vol128, 320, 180, fmt=vr.FMT_RGBA8_UNORM)
    assert img.dtype == np.uint8
    assert_exact(img, ref)
    img, ref, _, _ = render_both(r, oracle, vol128, 320, 180, fmt=vr.FMT_RGBA8_SRGB)
    assert np.abs(img.astype(int) - ref.astype(int)).max() <= 1


def test_band_sharding_and_assembly(r, oracle, vol128):
    W, H, br, n = 320, 200, 16, 3
    osd, gsd = vr.reference_shader_data(W / H, 15.0, 5.0)
    r.set_volume(vol128)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults())
    full = r.render(W, H, vr.FMT_RGBA32F)
    rows0 = vr.band_rows_packed(H, br, n, 0)
    gathered = torch.zeros((n, rows0, W, 4), dtype=torch.float32, device="cuda")
    total = 0
    for k in range(n):
        rows = vr.band_rows_packed(H, br, n, k)
        r.render(W, H, vr.FMT_RGBA32F, out=gathered[k, :rows], band_rows=br, band_stride=n, band_first=k)
        obj, glob = vr.shader_data_arrays(osd, gsd)
        ref, _ = oracle.render(vol128, obj, glob, oracle.march(), W, H, oracle.FMT_RGBA32F, band_rows=br,
                               band_stride=n, band_first=k)
        got = gathered[k, :rows].cpu().numpy()
        valid = [i for i in range(rows) if ((k + (i // br) * n) * br + i % br) < H]
        assert_exact(got[valid], ref[valid])
        total += rows
    frame = r.assemble_bands(gathered, n, W, H, br)
    torch.cuda.synchronize()
    assert_exact(frame.cpu().numpy(), full.cpu().numpy())


@pytest.mark.parametrize("fmt", [vr.FMT_RGBA32F, vr.FMT_RGBA8_UNORM, vr.FMT_RGBA8_SRGB] if torch.cuda.is_available()
                         else [])
def test_grey_targets_and_expanding_assembly(r, oracle, vol128, fmt):
    """Grey targets (include/vr.h formats 3-5) hold the R channel of the RGBA
    format bit for bit, for the grid and the procedural march, whole frames
    and band sets; grey band sets of 3 ranks, gathered and expanded by
    vr_assemble_frame, equal the RGBA frame (G = B = R, A = 1 / 255).  Widths
    320 and 203 take the 4-pixel and the per-pixel expansion."""
    g = vr.GREY_OF[fmt]
    r.set_volume(vol128)
    try:
        for proc in (False, True):
            if proc:
                r.set_procedural()
            for W, H in [(320, 200), (203, 117)]:
                osd, gsd = vr.reference_shader_data(W / H, 15.0, 5.0)
                r.set_shader_data(osd, gsd)
                r.set_march(vr.march_defaults(max_steps=64))
                full = r.render(W, H, fmt)
                grey = r.render(W, H, g)
                torch.cuda.synchronize()
                assert tuple(grey.shape) == (H, W)
                assert torch.equal(grey, full[..., 0])
                if not proc:
                    obj, glob = vr.shader_data_arrays(osd, gsd)
                    ref, _ = oracle.render(vol128, obj, glob, oracle.march(64), W, H, fmt)
                    assert_exact(grey.cpu().numpy(), np.ascontiguousarray(ref[..., 0]))
                br, n = 16, 3
                gathered = torch.zeros((n, vr.band_rows_packed(H, br, n, 0), W), dtype=grey.dtype, device="cuda")
                for k in range(n):
                    rows = vr.band_rows_packed(H, br, n, k)
                    r.render(W, H, g, out=gathered[k, :rows], band_rows=br, band_stride=n, band_first=k)
                frame = r.assemble_frame(gathered, g, n, W, H, br, fmt)
                same = r.assemble_frame(gathered, g, n, W, H, br, g)   # equal formats: a plain scatter
                torch.cuda.synchronize()
                assert_exact(frame.cpu().numpy(), full.cpu().numpy())
                assert torch.equal(same, grey)
        with pytest.raises(ValueError):
            r.assemble_frame(gathered, g, n, W, H, br, vr.GREY_OF[(fmt + 1) % 3])
    finally:
        r.set_procedural(enabled=0)


def serpentine_rows(H, br, stride, first, flip, rows):
    """Frame row of each of a band set's `rows` packed rows (vr.h
    vr_target.band_flip: band k is first + k*stride, + flip for odd k); -1
    past the frame."""
    out = []
    for j in range(rows):
        k = j // br
        y = (first + k * stride + (flip if k % 2 else 0)) * br + j % br
        out.append(y if y < H else -1)
    return np.array(out)


def test_serpentine_band_sets_and_assembly(r, oracle, vol128):
    """Band sets with flipped odd bands (vr_target.band_flip), as the
    multi-GPU loop deals them serpentine (vr_shard_set_serpentine): each of S
    renderers' sets (flip S-1-2i) holds its frame rows bit-exact against the
    oracle's frame, their step counts sum to the frame's, grey sets gathered
    and expanded with VR_ASSEMBLE_SERPENTINE equal the frame, and a set
    below a lead of rows (first = lead bands + i) and an in-place set land at
    their own rows.  Grid (regions and static schedules) and procedural media;
    band heights 16, 8 and 24, partial last bands."""
    import ctypes
    from volumetricrenderer_amd import _lib
    r.set_volume(vol128)
    cases = [(320, 200, 16, 3, False, -1), (333, 197, 8, 7, False, -1), (320, 200, 24, 2, False, 0),
             (200, 150, 16, 3, True, -1)]
    try:
        for W, H, br, S, proc, sched in cases:
            osd, gsd = vr.reference_shader_data(W / H, 15.0, 5.0)
            march = vr.march_defaults(max_steps=64)
            r.set_shader_data(osd, gsd)
            r.set_march(march)
            r.set_option("schedule", sched)
            obj, glob = vr.shader_data_arrays(osd, gsd)
            if proc:
                # (no shadow rays: a small frame's deferred-scratch need, per
                # pixel-step, would size the later 1080p frames' scratch)
                r.set_procedural(shadow_steps=0)
                ref, steps = oracle.render_procedural(oracle.procedural_from(r.procedural), obj, glob,
                                                      oracle.from_params(march), W, H, 0)
            else:
                r.set_procedural(enabled=0)
                ref, steps = oracle.render(vol128, obj, glob, oracle.march(64), W, H, oracle.FMT_RGBA32F)
            fmt, g = vr.FMT_RGBA32F, vr.GREY_OF[vr.FMT_RGBA32F]
            rows_max = max(vr.band_rows_packed(H, br, S, i, S - 1 - 2 * i) for i in range(S))
            gathered = torch.zeros((S, rows_max, W), dtype=torch.float32, device="cuda")
            total = 0
            for i in range(S):
                fl = S - 1 - 2 * i
                rows = vr.band_rows_packed(H, br, S, i, fl)
                cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
                out = r.alloc_target(W, H, fmt, br, S, i, fl)
                out.fill_(float("nan"))
                r.render(W, H, fmt, out=out, band_rows=br, band_stride=S, band_first=i, band_flip=fl, step_counter=cnt)
                r.render(W, H, g, out=gathered[i, :rows], band_rows=br, band_stride=S, band_first=i, band_flip=fl)
                torch.cuda.synchronize()
                total += int(cnt.item())
                ys = serpentine_rows(H, br, S, i, fl, rows)
                assert_exact(out.cpu().numpy()[ys >= 0], ref[ys[ys >= 0]])
            assert total == steps
            frame = r.assemble_frame(gathered, g, S, W, H, br, fmt, serpentine=True)
            torch.cuda.synchronize()
            assert_exact(frame.cpu().numpy(), ref)
            # below a lead of two bands: renderer i's set starts at band 2 + i
            lead = 2
            for i in range(S):
                fl = S - 1 - 2 * i
                out = r.render(W, H, fmt, band_rows=br, band_stride=S, band_first=lead + i, band_flip=fl)
                torch.cuda.synchronize()
                ys = serpentine_rows(H, br, S, lead + i, fl, out.shape[0])
                assert_exact(out.cpu().numpy()[ys >= 0], ref[ys[ys >= 0]])
            # in place: renderer S-1's rows at their frame rows, the rest untouched
            frame = r.alloc_target(W, H, fmt)
            frame.fill_(float("nan"))
            fl = S - 1 - 2 * (S - 1)
            t = _lib.Target(width=W, height=H, format=fmt | _lib.TARGET_BANDS_IN_PLACE, band_rows=br, band_stride=S,
                            band_first=S - 1, pixels=frame.data_ptr(), row_pitch=frame.stride(0) * frame.element_size(),
                            step_counter=None, band_flip=fl)
            _lib.call("vr_render", r._ctx, ctypes.byref(t), None)
            torch.cuda.synchronize()
            got = frame.cpu().numpy()
            mine = serpentine_rows(H, br, S, S - 1, fl, vr.band_rows_packed(H, br, S, S - 1, fl))
            mine = mine[mine >= 0]
            assert_exact(got[mine], ref[mine])
            assert np.isnan(np.delete(got, mine, axis=0)).all()
        buf = torch.zeros((64, 64, 4), device="cuda")
        for stride, flip, fmt in ((3, 3, 0), (3, -3, 0), (1, 1, 0), (3, 1, 0x200)):   # |flip| >= stride, row range
            t = _lib.Target(width=64, height=64, format=fmt, band_rows=16, band_stride=stride, band_first=0,
                            pixels=buf.data_ptr(), row_pitch=0, step_counter=None, band_flip=flip)
            with pytest.raises(vr.VRError):
                _lib.call("vr_render", r._ctx, ctypes.byref(t), None)
    finally:
        r.set_procedural(enabled=0)
        r.set_option("schedule", -1)


def test_volume_generator_matches_oracle(r, oracle):
    for literal in (True, False):
        rec = vr.volume_recipe_defaults(size=48, literal_overwrite=int(literal))
        r.generate_volume(rec)
        got = r.get_volume()
        ref = oracle.build_volume(48, literal=literal)
        assert_exact(got, ref)
        if literal:
            assert (got[..., 1] == got[0, 0, 0, 1]).all()  # G constant (TestMain.cpp:60, :76)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_noise_grid_matches_oracle(r, oracle, kind):
    out = torch.empty((20, 24, 28), dtype=torch.float32, device="cuda")
    _, mn, mx = r.noise_grid(kind, 28, 24, 20, 0.173, 77, origin=(-9, 5, 1000), out=out)
    ref, rmn, rmx = oracle.noise_grid(kind, 28, 24, 20, 0.173, 77, origin=(-9, 5, 1000))
    assert_exact(out.cpu().numpy(), ref)
    assert (mn, mx) == (rmn, rmx)


def test_random_cases(r, oracle):
    rng = np.random.default_rng(1234)
    for case in range(8):
        dims = tuple(int(x) for x in rng.integers(8, 80, size=3))
        vol = rng.integers(0, 256, size=dims[::-1] + (4,), dtype=np.uint8)
        W, H = int(rng.integers(17, 300)), int(rng.integers(9, 200))
        osd, gsd = vr.reference_shader_data(float(W) / H, float(rng.uniform(-180, 180)), float(rng.uniform(-90, 90)))
        m = vr.march_defaults(max_steps=int(rng.integers(1, 200)))
        img, ref, c, s = render_both(r, oracle, vol, W, H, osd, gsd, m)
        assert_exact(img, ref)
        assert c == s, case


def test_errors(oracle):
    with vr.Renderer(0) as rr:
        with pytest.raises(VRError) as e:
            rr.render(64, 64)
        assert e.value.status == 3  # VR_ERR_NO_VOLUME
        rr.set_volume(np.zeros((4, 4, 4, 4), np.uint8))
        with pytest.raises(VRError) as e:
            rr.render(64, 64)
        assert e.value.status == 4  # VR_ERR_NO_CAMERA
        osd, gsd = vr.reference_shader_data(1.0)
        gsd.camera_position[0] = 7.0  # not the View eye: accepted (frag.glsl:36-38)
        rr.set_shader_data(osd, gsd)
        with pytest.raises(ValueError):   # a target the kernel would write past
            rr.render(64, 64, vr.FMT_RGBA32F, out=torch.zeros((64, 64, 4), dtype=torch.uint8, device="cuda"))
        with pytest.raises(ValueError):
            rr.render(64, 64, vr.FMT_RGBA8_UNORM, out=torch.zeros((32, 64, 4), dtype=torch.uint8, device="cuda"))
        with pytest.raises(VRError):
            rr.set_march(vr.march_defaults(max_steps=0))
        with pytest.raises(ValueError):
            rr.set_volume(np.zeros((4, 4, 4), np.uint8))


def test_config5_grid512_bands(r, oracle):
    """BASELINE config 5: 512^3 recipe volume (GPU-generated), 1080p x 128.
    Checked against the oracle on every 24th 16-row band, plus determinism."""
    r.generate_volume(vr.scaled_recipe(512))
    vol = r.get_volume()
    osd, gsd = vr.reference_shader_data(16 / 9)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults())
    W, H = 1920, 1080
    a = r.render(W, H, vr.FMT_RGBA32F).cpu().numpy()
    b = r.render(W, H, vr.FMT_RGBA32F).cpu().numpy()
    assert_exact(a, b)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    for first in (0, 11, 17):
        ref, _ = oracle.render(vol, obj, glob, oracle.march(), W, H, oracle.FMT_RGBA32F, band_rows=16,
                               band_stride=24, band_first=first)
        rows = [(first + (i // 16) * 24) * 16 + i % 16 for i in range(ref.shape[0])]
        keep = [i for i, y in enumerate(rows) if y < H]
        assert_exact(a[[rows[i] for i in keep]], ref[keep])


def test_config1_matches_golden_fixture(r):
    """The HIP path against the committed config-1 frame (tests/golden)."""
    import os
    import sys
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, golden)
    from make_golden import perlin_cube_volume
    ref = np.load(os.path.join(golden, "config1_256x256x32.npy"))
    r.set_volume(perlin_cube_volume())
    osd, gsd = vr.reference_shader_data(1.0)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults(max_steps=32))
    img = r.render(256, 256, vr.FMT_RGBA32F).cpu().numpy()
    assert np.array_equal(img[..., 0], ref)


# ---- procedural medium (BASELINE configs 2/3; build-defined) ----

def render_proc_both(r, oracle, W, H, march, fmt=0, osd=None, gsd=None, schedule=-1, band=None, **proc):
    if osd is None:
        osd, gsd = vr.reference_shader_data(W / H, 20.0, 15.0)
    band = band or {}
    r.set_shader_data(osd, gsd)
    r.set_march(march)
    r.set_procedural(**proc)
    r.set_option("schedule", schedule)
    p = oracle.procedural_from(r.procedural)
    try:
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        img = r.render(W, H, fmt, step_counter=cnt, **band)
        torch.cuda.synchronize()
        variant = r.kernel_variant
    finally:
        r.set_procedural(enabled=0)
        r.set_option("schedule", -1)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    ref, steps = oracle.render_procedural(p, obj, glob,
                                          oracle.from_params(march), W, H, fmt, **band)
    return img.cpu().numpy(), ref, int(cnt.item()), steps, variant


@pytest.mark.parametrize("schedule,suffix", [(-1, ""), (0, "_tiles"), (4, "_rings")])
def test_procedural_config2_cloud(r, oracle, schedule, suffix):
    img, ref, c, s, var = render_proc_both(r, oracle, 192, 108, vr.march_defaults(max_steps=128), schedule=schedule)
    assert var == "procedural" + suffix
    assert_exact(img, ref)
    assert c == s > 0
    assert img[..., 0].max() > 0.05   # the cloud is not empty


@pytest.mark.parametrize("schedule,suffix", [(-1, ""), (0, "_tiles"), (4, "_rings")])
def test_procedural_config3_shadow(r, oracle, schedule, suffix):
    img, ref, c, s, var = render_proc_both(r, oracle, 128, 72, vr.march_defaults(max_steps=128), schedule=schedule,
                                           shadow_steps=8)
    assert var == "procedural_shadow" + suffix
    assert_exact(img, ref)
    assert c == s > 0
    assert img[..., 0].max() > 0.0


def test_procedural_shadow_region_enumeration(r, oracle):
    """Config 3 with the 64x64-region sort enumeration (option "proc_enum",
    a round-3 experiment; row-major is the default with shadow rays) stays
    bit-exact, with early-out and short shadow runs too."""
    need_experiments(r, "proc_enum")
    r.set_option("proc_enum", 1)
    try:
        for W, H, m, kw in [(128, 72, vr.march_defaults(max_steps=128), dict(shadow_steps=8)),
                            (96, 64, vr.march_defaults(max_steps=96, density=400.0, early_out=0.01),
                             dict(shadow_steps=5, sun_dir=(-1.0, 0.5, 0.25)))]:
            img, ref, c, s, var = render_proc_both(r, oracle, W, H, m, **kw)
            assert var == "procedural_shadow"
            assert_exact(img, ref)
            assert c == s > 0
    finally:
        r.set_option("proc_enum", 0)


DEFER_CASES = [
    (128, 72, dict(max_steps=128), dict(shadow_steps=8), {}),
    (96, 64, dict(max_steps=96, density=400.0, early_out=0.01), dict(shadow_steps=5, sun_dir=(-1.0, 0.5, 0.25)), {}),
    (96, 64, dict(max_steps=48, density=3.0), dict(shadow_steps=21, sun_dir=(0.3, -1.0, 2.0)), {}),
    (96, 64, dict(max_steps=48, density=3.0), dict(shadow_steps=8, sun_dir=(0.0, 0.0, -1.0)), {}),
    (96, 64, dict(max_steps=48, density=3.0), dict(shadow_steps=1, octaves=6, gain=0.6), {}),
    (200, 150, dict(max_steps=64), dict(shadow_steps=8), dict(band_rows=16, band_stride=3, band_first=1)),
    (1, 1, dict(max_steps=64), dict(shadow_steps=8), {}),
    (67, 9, dict(max_steps=64), dict(shadow_steps=8), {}),
]


@pytest.mark.parametrize("case", range(len(DEFER_CASES)))
def test_procedural_shadow_deferred(r, oracle, case):
    """Deferred shadow rays (option "shadow_defer": primary march appends
    (P, coefficient) entries, one thread per entry sums its sun samples, a
    resolve pass folds them per ray in step order): bit-exact against the
    oracle and equal to the in-wave compaction, with step counts (count 0),
    density evaluations (count 1) and Worley cells (count 2); shadow runs
    longer than the compaction's limit, early-out, zero sun components, bands
    and frames smaller than a wave."""
    W, H, m, kw, band = DEFER_CASES[case]
    march = vr.march_defaults(**m)
    imgs, counts = [], []
    try:
        for defer, cache in ((1, 0), (0, 0), (1, 1), (1, 2)):   # shadow pass: register Worley cube / 8 lanes per entry
            r.set_option("shadow_defer", defer)
            r.set_option("shadow_cache", cache)
            img, ref, c, s, var = render_proc_both(r, oracle, W, H, march, band=band, **kw)
            assert var == "procedural_shadow"
            assert_exact(img, ref)
            assert c == s
            imgs.append(img)
            cc = []
            for cm in (1, 2):
                r.set_option("count", cm)
                img2, _, c2, _, _ = render_proc_both(r, oracle, W, H, march, band=band, **kw)
                cc.append(c2)
                assert np.array_equal(img2, img)
            r.set_option("count", 0)
            counts.append(cc)
    finally:
        r.set_option("shadow_defer", 1)   # the default
        r.set_option("shadow_cache", 0)
        r.set_option("count", 0)
    for k in range(1, len(imgs)):
        assert np.array_equal(imgs[0], imgs[k]), k
        assert counts[0] == counts[k], k


def test_procedural_shadow_deferred_scratch_limit(r, oracle):
    """The deferred-shadow scratch is sized from the frame (vr_api.cpp
    ensure_defer): sorted wave w owns the entry range proc_scan lays out from
    the cost histogram, and a wave past the capacity marches its shadow rays in
    place.  Exact with a capacity of 4096 entries (most waves in place), with
    the frame-sized scratch, and with shadow_defer_mib 0 (no scratch: the
    in-wave compaction) -- the same frame every time."""
    W, H = 128, 72
    march = vr.march_defaults(max_steps=128)
    assert r.get_option("shadow_defer_mib") == 4096
    imgs = []
    try:
        for ents, mib in ((4096, 4096), (0, 4096), (0, 0)):
            r.set_option("shadow_defer_entries", ents)
            r.set_option("shadow_defer_mib", mib)
            img, ref, c, s, _ = render_proc_both(r, oracle, W, H, march, shadow_steps=8)
            assert_exact(img, ref)
            assert c == s
            assert r.get_option("shadow_defer_last") == (1 if mib else 0)
            kib = r.get_option("shadow_defer_kib")
            assert (0 < kib < 4096) if mib else kib == 0
            imgs.append(img)
    finally:
        r.set_option("shadow_defer_entries", 0)
        r.set_option("shadow_defer_mib", 4096)
    assert np.array_equal(imgs[0], imgs[1]) and np.array_equal(imgs[0], imgs[2])


def proc_frame_bands(r, oracle, W, H, march, firsts, stride=24, fmt=0, **proc):
    """A whole procedural frame on the GPU against the oracle on interleaved
    16-row band subsets, and its executed-step count against the oracle's
    geometry (frag.glsl:46).  Returns the GPU frame."""
    osd, gsd = vr.reference_shader_data(16 / 9)
    r.set_shader_data(osd, gsd)
    r.set_march(march)
    r.set_procedural(**proc)
    p = oracle.procedural_from(r.procedural)
    try:
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        img = r.render(W, H, fmt, step_counter=cnt).cpu().numpy()
        defer = r.get_option("shadow_defer_last")
        kib = r.get_option("shadow_defer_kib")
    finally:
        r.set_procedural(enabled=0)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    for first in firsts:
        ref, _ = oracle.render_procedural(p, obj, glob, oracle.from_params(march), W, H, fmt, band_rows=16,
                                          band_stride=stride, band_first=first)
        rows = [(first + (i // 16) * stride) * 16 + i % 16 for i in range(ref.shape[0])]
        keep = [i for i, y in enumerate(rows) if y < H]
        assert_exact(img[[rows[i] for i in keep]], ref[keep])
    n = oracle.step_counts(obj, glob, oracle.from_params(march), W, H)
    assert int(cnt.item()) == int(n[n > 0].sum(dtype=np.int64))
    return img, defer, kib


def test_config3_full_frame_bands(r, oracle):
    """BASELINE config 3 at its full shape: the whole 1920x1080x128 frame with
    8-step shadow rays, on the deferred passes (12,150 shadow workgroups),
    against the oracle on three interleaved band subsets, with the whole-frame
    step count.  Rendered twice: the second frame runs with the scratch sized
    from the first one's need, <= 0.4 GB (the old per-wave worst case took
    4.2 GB)."""
    march = vr.march_defaults(max_steps=128)
    for rep in range(2):
        img, defer, kib = proc_frame_bands(r, oracle, 1920, 1080, march, (0, 11, 17) if rep else (5,),
                                           shadow_steps=8)
        assert defer == 1
        assert 0 < kib <= 400 * 1024, kib
        assert img[..., 0].max() > 0.05


def test_config3_4k_256_deferred(r, oracle):
    """Config 3's medium at config 4's shape (3840x2160, 256 steps): the frame
    takes the deferred path (its worst-case scratch would have been ~68 GB),
    exact against the oracle on band subsets, with the whole-frame step
    count."""
    march = vr.march_defaults(max_steps=256)
    img, defer, kib = proc_frame_bands(r, oracle, 3840, 2160, march, (3, 40), stride=48, shadow_steps=8)
    assert defer == 1
    assert 0 < kib <= 4096 * 1024


def test_procedural_shadow_deferred_stale_and_reuse(r, oracle):
    """The deferred passes with a reused sort order (background fill blocks)
    and a stale one (option sort_reuse: leftover pixels marched inline by the
    trailing blocks), over a spinning camera: exact every frame."""
    W, H = 160, 90
    march = vr.march_defaults(max_steps=64)
    r.set_option("shadow_defer", 1)
    need_experiments(r, "sort_reuse")
    r.set_option("sort_reuse", 2)
    try:
        for k, phi in enumerate([20.0, 20.0, 21.6, 23.2, 24.8, 24.8]):
            osd, gsd = vr.reference_shader_data(W / H, phi, 15.0)
            img, ref, c, s, _ = render_proc_both(r, oracle, W, H, march, osd=osd, gsd=gsd, shadow_steps=8)
            assert_exact(img, ref)
            assert c == s, k
    finally:
        r.set_option("shadow_defer", 1)
        r.set_option("sort_reuse", 0)


@pytest.mark.parametrize("kw", [dict(octaves=1, seed_fbm=11), dict(octaves=6, gain=0.6, worley_freq=0.05),
                                dict(shadow_steps=3, sun_dir=(0.0, 1.0, 0.0)),
                                dict(shadow_steps=16, sun_dir=(-1.0, 0.5, 0.25)),
                                dict(shadow_steps=21, sun_dir=(0.3, -1.0, 2.0)),     # > compaction limit
                                dict(shadow_steps=8, sun_dir=(0.0, 0.0, -1.0)),      # in-box runs, zero components
                                dict(shadow_steps=7, sun_dir=(-1.0, -1.0, 0.2), freq0=0.31),
                                dict(shadow_steps=5, schedule=0),
                                dict(worley_freq=0.1),                   # cell table too big: direct noise
                                dict(worley_freq=-0.02, grid_scale=200.0, shadow_steps=4),
                                dict(octaves=0)])
def test_procedural_parameters(r, oracle, kw):
    img, ref, c, s, _ = render_proc_both(r, oracle, 96, 64, vr.march_defaults(max_steps=48, density=3.0), **kw)
    assert_exact(img, ref)
    assert c == s


@pytest.mark.parametrize("shadow", [0, 4])
def test_procedural_early_out_and_rgba8(r, oracle, shadow):
    m = vr.march_defaults(max_steps=96, density=400.0, early_out=0.01)
    img, ref, c, s, _ = render_proc_both(r, oracle, 96, 64, m, fmt=vr.FMT_RGBA8_UNORM, shadow_steps=shadow)
    assert_exact(img, ref)
    assert c == s
    full = vr.march_defaults(max_steps=96, density=400.0)
    _, _, c2, _, _ = render_proc_both(r, oracle, 96, 64, full, fmt=vr.FMT_RGBA8_UNORM, shadow_steps=shadow)
    assert c < c2   # the early-out really skipped steps


def test_procedural_sort_reuse(r, oracle):
    """The cost-sorted order is reused while the frame geometry is unchanged
    (vr_api.cpp sort key) -- across medium changes -- and rebuilt when the
    camera, band set or shadow flag changes.  Each render goes into a target
    prefilled with garbage, so a reused order must still write every pixel
    (the background fill).  Exact against the oracle every time."""
    W, H = 160, 90
    march = vr.march_defaults(max_steps=48)
    cams = [vr.reference_shader_data(W / H, 20.0, 15.0), vr.reference_shader_data(W / H, -40.0, 5.0)]
    seq = [(0, {}, dict(octaves=4)), (0, {}, dict(octaves=3, seed_fbm=7)), (1, {}, dict(octaves=4)),
           (0, {}, dict(octaves=4, shadow_steps=8)), (0, {}, dict(octaves=2, shadow_steps=8)),
           (0, dict(band_rows=16, band_stride=2, band_first=1), dict(octaves=4)),
           (0, dict(band_rows=16, band_stride=2, band_first=1), dict(octaves=4, seed_fbm=11)),
           (0, {}, dict(octaves=4))]
    for cam, band, proc in seq:
        osd, gsd = cams[cam]
        r.set_shader_data(osd, gsd)
        r.set_march(march)
        r.set_procedural(**proc)
        try:
            out = r.alloc_target(W, H, vr.FMT_RGBA32F, **band)
            out.fill_(123.0)
            r.render(W, H, vr.FMT_RGBA32F, out=out, **band)
            torch.cuda.synchronize()
            p = oracle.procedural_from(r.procedural)
        finally:
            r.set_procedural(enabled=0)
        obj, glob = vr.shader_data_arrays(osd, gsd)
        ref, _ = oracle.render_procedural(p, obj, glob, oracle.from_params(march), W, H, 0, **band)
        # packed rows that map past the frame (a partial last band) are not
        # written (vr.h vr_target); compare the frame's rows
        rows = np.arange(out.shape[0])
        if band:
            bl = rows // band["band_rows"]
            rows = rows[(band["band_first"] + bl * band["band_stride"]) * band["band_rows"]
                        + rows % band["band_rows"] < H]
        assert_exact(out.cpu().numpy()[rows], ref[rows])


@pytest.mark.parametrize("shadow", [0, 8])
def test_procedural_bands(r, oracle, shadow):
    band = dict(band_rows=16, band_stride=3, band_first=1)
    img, ref, c, s, _ = render_proc_both(r, oracle, 200, 150, vr.march_defaults(max_steps=64), band=band,
                                         shadow_steps=shadow)
    assert_exact(img, ref)
    assert c == s


def test_procedural_1080p_config2_full_frame(r, oracle):
    """BASELINE config 2 at its full size (the oracle takes a few seconds)."""
    osd, gsd = vr.reference_shader_data(1280.0 / 720.0)
    img, ref, c, s, _ = render_proc_both(r, oracle, 1920, 1080, vr.march_defaults(), fmt=vr.FMT_RGBA8_UNORM,
                                         osd=osd, gsd=gsd)
    assert_exact(img, ref)
    assert c == s == 16737882


@pytest.mark.parametrize("kw", [dict(), dict(freq0=-0.23, octaves=3), dict(lacunarity=-1.7, octaves=5, seed_fbm=5),
                                dict(octaves=9), dict(shadow_steps=8)])
def test_procedural_lattice_table(r, oracle, kw):
    """The Perlin lattice table (vr_api.cpp ensure_lattice, option
    "lattice"): exact against the oracle with it and without it, for negative
    frequencies (cells below 0), alternating-sign lacunarity, a range too
    large for the table (9 octaves: the per-octave hash path) and shadows."""
    march = vr.march_defaults(max_steps=64)
    try:
        imgs = []
        for lat in (1, 0):
            r.set_option("lattice", lat)
            img, ref, c, s, _ = render_proc_both(r, oracle, 112, 80, march, **kw)
            assert_exact(img, ref)
            assert c == s
            imgs.append(img)
        assert np.array_equal(imgs[0], imgs[1])
    finally:
        r.set_option("lattice", 1)


def test_procedural_rejects_bad_parameters(r):
    with pytest.raises(VRError):
        r.set_procedural(octaves=17)
    with pytest.raises(VRError):
        r.set_procedural(shadow_steps=8, sun_dir=(0.0, 0.0, 0.0))
    r.set_procedural(enabled=0)


def test_procedural_density_evaluation_count(r, oracle):
    """count=1: the step counter sums density evaluations (ray-steps + shadow
    samples), the unit of bench.py's procedural roofline."""
    W, H = 96, 64
    m = vr.march_defaults(max_steps=64)
    osd, gsd = vr.reference_shader_data(W / H, 20.0, 15.0)
    r.set_shader_data(osd, gsd)
    r.set_march(m)
    r.set_procedural(shadow_steps=8)
    p = oracle.procedural_from(r.procedural)
    r.set_option("count", 1)
    got = []
    try:
        for sched in (-1, 0):
            r.set_option("schedule", sched)
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            r.render(W, H, 0, step_counter=cnt)
            torch.cuda.synchronize()
            got.append(int(cnt.item()))
    finally:
        r.set_option("count", 0)
        r.set_option("schedule", -1)
        r.set_procedural(enabled=0)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    _, steps, evals = oracle.render_procedural(p, obj, glob,
                                               oracle.from_params(m), W, H, 0, with_evals=True)
    assert got == [evals, evals] and evals > steps


@pytest.mark.parametrize("shadow", [0, 8])
def test_procedural_worley_cell_count(r, oracle, shadow):
    """count=2: the step counter sums the Worley cells the pruned evaluation
    really computed (8 per sample, 35 when the 27-cell block also ran) -- the
    per-sample work bench.py's procedural roofline counts (verdict r02 #2).
    The oracle mirrors the pruning decision with a correctly rounded square
    root where the device uses v_sqrt_f32, so a sample whose test sits within
    an ulp of the bound may count 27 cells differently: the bar is 1e-5 of
    the total.  The plain-tile schedule (schedule 0) evaluates F1 from the
    unpruned cell table: exactly 27 cells per evaluation."""
    W, H = 160, 96
    m = vr.march_defaults(max_steps=128)
    osd, gsd = vr.reference_shader_data(W / H, -15.0, 25.0)
    r.set_shader_data(osd, gsd)
    r.set_march(m)
    r.set_procedural(shadow_steps=shadow)
    p = oracle.procedural_from(r.procedural)
    got = []
    try:
        for sched in (-1, 0):
            r.set_option("schedule", sched)
            r.set_option("count", 2)
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            r.render(W, H, 0, step_counter=cnt)
            r.set_option("count", 1)
            ev = torch.zeros(1, dtype=torch.int64, device="cuda")
            r.render(W, H, 0, step_counter=ev)
            torch.cuda.synchronize()
            got.append((int(cnt.item()), int(ev.item())))
    finally:
        r.set_option("count", 0)
        r.set_option("schedule", -1)
        r.set_procedural(enabled=0)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    _, steps, evals, cells = oracle.render_procedural(p, obj, glob, oracle.from_params(m), W, H, 0,
                                                      with_evals=True, with_cells=True)
    assert got[0][1] == got[1][1] == evals
    cells_sorted, cells_tiles = got[0][0], got[1][0]
    assert cells_tiles == 27 * evals
    assert abs(cells_sorted - cells) <= max(27, 1e-5 * cells), (cells_sorted, cells)
    assert 8 * evals <= cells <= 35 * evals
    assert cells < 12 * evals   # pruning keeps the mean far below 27 cells per sample


def test_cellular_inv_shortcut_exhaustive(r):
    """The cellular cell-point magnitude the noise kernels use equals
    jitter / sqrtf(d2) (IEEE) on every input of its domain."""
    assert r.selftest("cell_inv") == 0
    with pytest.raises(VRError):
        r.selftest("nope")


def test_worley_pruning_bit_exact(r):
    """The pruned Worley F1 of the procedural march (8-cell cube, the other
    19 cells only when the distance bound needs them) equals the full
    27-cell cellular() bit for bit on 2^23 points per seed, including points
    a few ulps around the rint / floor switches, at feature points and
    between two of them (vr_selftest "worley_prune")."""
    assert r.selftest("worley_prune") == 0


def translated_shader_data(W, H, t):
    """Reference camera with Model = translate(t) and W2L = its inverse, so the
    projected box centre leaves the screen centre (ring schedule centring)."""
    import ctypes
    osd, gsd = vr.reference_shader_data(W / H)
    obj, glob = vr.shader_data_arrays(osd, gsd)
    obj[12:15] = np.float32(t)
    glob[12:15] = -np.float32(t)
    ctypes.memmove(ctypes.byref(osd), obj.ctypes.data, obj.nbytes)
    ctypes.memmove(ctypes.byref(gsd), glob.ctypes.data, glob.nbytes)
    return osd, gsd


@pytest.mark.parametrize("t", [(0.9, -0.4, 0.2), (1.8, -1.8, 0.0), (0.0, 0.0, 3.5)])
@pytest.mark.parametrize("layout", [15, 5])
@pytest.mark.parametrize("schedule", [4, 5])
def test_ring_schedule_off_centre(r, oracle, vol128, t, layout, schedule):
    W, H = 400, 240
    osd, gsd = translated_shader_data(W, H, t)
    r.set_layout_preference(layout)
    r.set_option("schedule", schedule)
    try:
        for band in ({}, dict(band_rows=16, band_stride=2, band_first=1)):
            img, ref, c, s = render_both(r, oracle, vol128, W, H, osd, gsd, **band)
            assert_exact(img, ref)
            assert c == s
    finally:
        r.set_option("schedule", -1)
        r.set_layout_preference(0)


@pytest.mark.parametrize("shadow,name", [(0, "config2_crop64"), (8, "config3_crop64")])
def test_procedural_matches_golden_crops(r, shadow, name):
    """The HIP path against the committed config-2/3 crops (tests/golden)."""
    import os
    import sys
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, golden)
    from make_golden import CROP_BAND, CROP_COLS
    ref = np.load(os.path.join(golden, name + ".npy"))
    osd, gsd = vr.reference_shader_data(1280.0 / 720.0)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults())
    r.set_procedural(shadow_steps=shadow)
    try:
        img = r.render(1920, 1080, vr.FMT_RGBA32F, **CROP_BAND).cpu().numpy()
    finally:
        r.set_procedural(enabled=0)
    assert np.array_equal(img[:, CROP_COLS[0]:CROP_COLS[1], 0], ref)


@pytest.mark.parametrize("procedural", [False, True])
def test_render_is_graph_capturable(r, vol128, procedural):
    """vr_render neither allocates nor synchronises once warm, so a frame can
    be captured in a hipGraph (torch.cuda.CUDAGraph) and replayed."""
    W, H = 320, 200
    osd, gsd = vr.reference_shader_data(W / H, 10.0, 5.0)
    r.set_volume(vol128)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults(max_steps=64))
    if procedural:
        r.set_procedural()
    try:
        out = r.alloc_target(W, H, vr.FMT_RGBA8_UNORM)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            r.render(W, H, vr.FMT_RGBA8_UNORM, out=out, stream=s)   # warm-up (allocates scratch)
        torch.cuda.synchronize()
        ref = out.clone()
        out.zero_()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            r.render(W, H, vr.FMT_RGBA8_UNORM, out=out, stream=s)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    finally:
        r.set_procedural(enabled=0)


def test_prepared_launchers_match_render(r, vol128):
    """prepare_render / prepare_assemble (the multi-GPU frame loop's fixed
    launchers) give the same pixels as render / assemble_bands."""
    W, H, nr, br = 300, 170, 3, 16
    osd, gsd = vr.reference_shader_data(W / H, 30.0, 10.0)
    r.set_volume(vol128)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults(max_steps=96))
    rows = vr.band_rows_packed(H, br, nr, 0)
    g = torch.zeros((nr, rows, W, 4), dtype=torch.uint8, device="cuda")
    for k in range(nr):
        r.prepare_render(W, H, vr.FMT_RGBA8_UNORM, g[k], band_rows=br, band_stride=nr, band_first=k)()
    frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    r.prepare_assemble(g, nr, W, H, br, frame)()
    full = r.render(W, H, vr.FMT_RGBA8_UNORM)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)


def test_procedural_needs_no_volume(oracle):
    """A context that never had a volume renders the procedural medium; with
    the medium off it reports VR_ERR_NO_VOLUME."""
    with vr.Renderer(0) as fresh:
        osd, gsd = vr.reference_shader_data(1.0)
        fresh.set_shader_data(osd, gsd)
        fresh.set_march(vr.march_defaults(max_steps=32))
        fresh.set_procedural()
        p = oracle.procedural_from(fresh.procedural)
        img = fresh.render(64, 64, vr.FMT_RGBA32F).cpu().numpy()
        obj, glob = vr.shader_data_arrays(osd, gsd)
        ref, _ = oracle.render_procedural(p, obj, glob, oracle.march(32), 64, 64, 0)
        assert_exact(img, ref)
        fresh.set_procedural(enabled=0)
        with pytest.raises(VRError) as e:
            fresh.render(64, 64, vr.FMT_RGBA32F)
        assert e.value.status == 3   # VR_ERR_NO_VOLUME


@pytest.mark.parametrize("wedges", [1, 3, 64])
def test_regions_schedule_every_pixel_once(r, oracle, vol128, wedges):
    """Regions schedule (5): the host-built per-XCD tile lists cover every
    tile exactly once -- the output buffer is pre-filled with a sentinel --
    and they are rebuilt when the geometry changes (camera, size, bands)."""
    W, H = 328, 200
    r.set_option("schedule", 5)
    r.set_option("wedges", wedges)
    try:
        r.set_volume(vol128)
        r.set_march(vr.march_defaults())
        cases = [(W, H, vr.reference_shader_data(W / H), {}),
                 (W, H, vr.reference_shader_data(W / H, 40.0, -25.0), {}),
                 (W + 40, H - 8, vr.reference_shader_data(W / H, 40.0, -25.0), {}),
                 (W, H, translated_shader_data(W, H, (1.1, -0.7, 0.3)), dict(band_rows=16, band_stride=3, band_first=1))]
        for w, h, (osd, gsd), band in cases:
            r.set_shader_data(osd, gsd)
            out = r.alloc_target(w, h, vr.FMT_RGBA8_UNORM, band.get("band_rows", 0), band.get("band_stride", 1),
                                 band.get("band_first", 0))
            out.fill_(0x5A)
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            img = r.render(w, h, vr.FMT_RGBA8_UNORM, out=out, step_counter=cnt, **band)
            torch.cuda.synchronize()
            obj, glob = vr.shader_data_arrays(osd, gsd)
            ref, steps = oracle.render(vol128, obj, glob, oracle.from_params(vr.march_defaults()), w, h,
                                       vr.FMT_RGBA8_UNORM, **band)
            assert_exact(img.cpu().numpy(), ref)
            assert int(cnt.item()) == steps
    finally:
        r.set_option("schedule", -1)
        r.set_option("wedges", 0)  # back to auto (vr_ctx.h wedges_of)


def test_regions_lists_across_streams(r, oracle, vol128):
    """Region lists built (and uploaded) on one stream and used on another,
    and rebuilt while both streams have queued renders: every frame exact."""
    r.set_option("schedule", 5)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        r.set_volume(vol128)
        r.set_march(vr.march_defaults())
        outs = []
        for i, (w, h) in enumerate([(200, 120), (200, 120), (232, 120), (232, 120), (200, 136), (200, 120)]):
            osd, gsd = vr.reference_shader_data(w / h, 15.0 * i, 5.0 * i)
            r.set_shader_data(osd, gsd)
            st = s1 if i % 2 == 0 else s2
            out = r.alloc_target(w, h, vr.FMT_RGBA8_UNORM)
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                out.fill_(0x33)
                r.render(w, h, vr.FMT_RGBA8_UNORM, out=out, stream=st)
            outs.append((w, h, osd, gsd, out))
        torch.cuda.synchronize()
        for w, h, osd, gsd, out in outs:
            obj, glob = vr.shader_data_arrays(osd, gsd)
            ref, _ = oracle.render(vol128, obj, glob, oracle.from_params(vr.march_defaults()), w, h,
                                   vr.FMT_RGBA8_UNORM)
            assert_exact(out.cpu().numpy(), ref)
    finally:
        r.set_option("schedule", -1)


@pytest.mark.parametrize("layout", [6, 7, 8, 9, 10, 11, 12, 13, 5, 14, 15])
@pytest.mark.parametrize("split", [2, 4, 8])
def test_split_rays_bitexact(r, oracle, vol128, layout, split):
    """Step-split rays (K lanes per ray, terms summed in step order): exact
    against the oracle, step counts included, with bands, a rotated cube,
    early-out and short rays (max_steps 7)."""
    if layout in EXPERIMENTAL_LAYOUTS:
        need_experiments(r, f"layout {layout}")
    r.set_layout_preference(layout)
    r.set_option("schedule", 5)
    r.set_option("split", split)
    try:
        osd, gsd = vr.reference_shader_data(16 / 9, 25.0, -40.0)
        for W, H, band, march in [(333, 187, {}, vr.march_defaults()),
                                  (640, 360, dict(band_rows=16, band_stride=3, band_first=2), vr.march_defaults()),
                                  (320, 180, {}, vr.march_defaults(max_steps=7)),
                                  (320, 180, {}, vr.march_defaults(early_out=0.6, density=4.0))]:
            img, ref, c, s = render_both(r, oracle, vol128, W, H, osd, gsd, march=march, **band)
            assert_exact(img, ref)
            assert c == s
    finally:
        r.set_option("split", 0)
        r.set_option("schedule", -1)
        r.set_layout_preference(0)


@pytest.mark.parametrize("layout", [15, 12, 5, 14])
def test_auto_split_at_one_eighth_band_share(r, oracle, vol128, layout):
    """The multi-GPU config-5 path: auto split (split=0) turns on for a 1/8
    band share of a 1080p frame, with col48 (the auto
    layout past the Infinity Cache since round 3), brick4832 (before it),
    corner8 and cornerh (the auto layout for cache-resident volumes).  Exact,
    step counts too."""
    r.set_layout_preference(layout)
    r.set_option("schedule", 5)
    r.set_option("split", 0)
    try:
        osd, gsd = vr.reference_shader_data(16 / 9)
        for first in (0, 5):
            img, ref, c, s = render_both(r, oracle, vol128, 1920, 1080, osd, gsd,
                                         band_rows=16, band_stride=8, band_first=first)
            assert_exact(img, ref)
            assert c == s
    finally:
        r.set_option("schedule", -1)
        r.set_layout_preference(0)


@pytest.mark.parametrize("order", [0, 1, 2])
@pytest.mark.parametrize("layout", [15, 14])
def test_region_order_bitexact(r, oracle, vol128, layout, order):
    """Option region_order: each XCD's list inside-out
    (0), longest tile first (1) or longest S x S block first (2, the
    default).  The lists only order the work: full frame, a 1/8 band share
    and GPU-rebuilt lists under a moving camera stay exact, step counts
    included."""
    r.set_layout_preference(layout)
    r.set_option("region_order", order)
    assert r.get_option("region_order") == order
    try:
        osd, gsd = vr.reference_shader_data(16 / 9, 20.0, -15.0)
        # band_first 3 of 8 holds the partial last band (frame rows 1072-1079):
        # its rows past the frame are left untouched (vr.h), so they are not compared
        for W, H, band in [(640, 360, {}), (1920, 1080, dict(band_rows=16, band_stride=8, band_first=3))]:
            img, ref, c, s = render_both(r, oracle, vol128, W, H, osd, gsd, **band)
            rows = sum(min(16, H - b * 16) for b in range(3, (H + 15) // 16, 8)) if band else H
            assert_exact(img[:rows], ref[:rows])
            assert c == s
        r.set_option("region_interval", 1)   # GPU rebuilds every render
        builds0 = r.get_option("region_gpu_builds")
        for i in range(1, 5):
            osd, gsd = vr.reference_shader_data(16 / 9, 20.0 + SPIN_DEG * i, -15.0)
            img, ref, c, s = render_both(r, oracle, vol128, 640, 360, osd, gsd)
            assert_exact(img, ref)
            assert c == s
        assert r.get_option("region_gpu_builds") - builds0 >= 3
    finally:
        r.set_option("region_interval", 32)
        r.set_option("region_order", 2)
        r.set_layout_preference(0)


@pytest.mark.parametrize("fmt", [0, 1, 3])   # RGBA32F, RGBA8_UNORM, R8_UNORM
def test_empty_tiles_filled_not_marched(r, oracle, vol128, fmt):
    """Option empty_fill (default 1): the regions lists put the tiles no ray
    of which can meet the box (vr_internal.h tile_is_empty: the box in front of
    the eye and outside one side plane of the tile's pixel-edge frustum) last,
    and the march writes them with the uncovered value instead of marching
    them.  Every pixel must come out as the full march writes it: the same
    bytes with the option on and off (targets pre-filled with a sentinel, so a
    pixel either run skips shows), across rotated models, bands (8- and 16-row;
    12-row bands are never classified), and GPU-built lists; and the oracle
    for two of them."""
    r.set_volume(vol128)
    r.set_march(vr.march_defaults())
    views = [(0.0, 0.0), (20.0, -15.0), (45.0, 30.0), (90.0, 0.0), (200.0, 60.0), (300.0, -80.0)]
    cases = [(640, 360, {}), (1920, 1080, dict(band_rows=16, band_stride=8, band_first=3)),
             (333, 197, dict(band_rows=8, band_stride=3, band_first=1)),
             (500, 300, dict(band_rows=12, band_stride=2, band_first=0))]
    seen_empty = 0
    r.set_option("region_interval", 1)   # lists for every camera (stale lists are marched whole)
    try:
        for phi, theta in views:
            for W, H, band in cases:
                osd, gsd = vr.reference_shader_data(W / H, phi, theta)
                r.set_shader_data(osd, gsd)
                outs = []
                for fill in (1, 0):
                    r.set_option("empty_fill", fill)
                    out = r.alloc_target(W, H, fmt, **band)
                    out.view(torch.uint8).fill_(0x5A)
                    r.render(W, H, fmt, out=out, **band)
                    torch.cuda.synchronize()
                    if fill:
                        e = r.get_option("region_empty_tiles")
                        seen_empty += max(e, 0)
                        if band.get("band_rows", 0) == 12:
                            assert e == 0
                    outs.append(out.cpu().numpy())
                assert_exact(outs[0], outs[1])
        assert seen_empty > 0
        r.set_option("empty_fill", 1)
        fmt = fmt if fmt in (0, 1) else 1   # the oracle renders RGBA (grey = R: test_grey_targets_*)
        for phi, theta in [(0.0, 0.0), (45.0, 30.0)]:
            osd, gsd = vr.reference_shader_data(16 / 9, phi, theta)
            img, ref, c, st = render_both(r, oracle, vol128, 640, 360, osd, gsd, fmt=fmt)
            assert_exact(img, ref)
            assert c == st
        for i in range(1, 4):   # GPU-built lists every render
            osd, gsd = vr.reference_shader_data(16 / 9, 20.0 + 7 * SPIN_DEG * i, -15.0)
            img, ref, c, st = render_both(r, oracle, vol128, 640, 360, osd, gsd, fmt=fmt)
            assert_exact(img, ref)
            assert c == st
        torch.cuda.synchronize()
        img, ref, c, st = render_both(r, oracle, vol128, 640, 360, osd, gsd, fmt=fmt)   # sized from the build
        assert_exact(img, ref)
        assert r.get_option("region_empty_tiles") > 0
    finally:
        r.set_option("region_interval", 32)
        r.set_option("empty_fill", 1)


# ---- BASELINE config 4: 3840x2160, 256 steps, 128^3 recipe volume ----

@pytest.fixture(scope="module")
def config4(r):
    """The config-4 frame at its stated shape on the HIP path: the 128^3
    reference-recipe volume generated on the GPU, reference camera (16:9),
    max_steps 256 (frag.glsl:30,42,46: step 1/64, at most 221 steps)."""
    r.generate_volume(vr.volume_recipe_defaults())
    vol = r.get_volume()
    osd, gsd = vr.reference_shader_data(16 / 9)
    march = vr.march_defaults(max_steps=256)
    return vol, osd, gsd, march


@pytest.mark.parametrize("fmt", [0, 1])
def test_config4_4k_256_bands(r, oracle, config4, fmt):
    """3840x2160x256, RGBA32F and RGBA8: the whole GPU frame against the
    oracle on three interleaved band subsets (every 24th 16-row band), and
    the executed-step count of the whole frame (1.348e8)."""
    vol, osd, gsd, march = config4
    W, H = 3840, 2160
    r.set_volume(vol)
    r.set_shader_data(osd, gsd)
    r.set_march(march)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    img = r.render(W, H, fmt, step_counter=cnt).cpu().numpy()
    steps = int(cnt.item())
    assert 134_000_000 < steps < 135_600_000
    obj, glob = vr.shader_data_arrays(osd, gsd)
    for first in (0, 13, 23):
        ref, _ = oracle.render(vol, obj, glob, oracle.from_params(march), W, H, fmt, band_rows=16,
                               band_stride=24, band_first=first)
        rows = [(first + (i // 16) * 24) * 16 + i % 16 for i in range(ref.shape[0])]
        keep = [i for i, y in enumerate(rows) if y < H]
        assert_exact(img[[rows[i] for i in keep]], ref[keep])
    # the whole-frame step count equals the oracle's (a3 truncation, frag.glsl:46)
    n = oracle.step_counts(obj, glob, oracle.from_params(march), W, H)
    assert steps == int(n[n > 0].sum(dtype=np.int64))


def test_config4_8_rank_loopback(r, config4):
    """Config 4 through the native 8-rank frame loop in loopback (every rank's
    interleaved band set rendered on this GPU into its gather slot, then
    vr_assemble_bands): the assembled frame equals a plain render -- with the
    defaults (serpentine band sets below rank 0's lead rows) and with row
    ranges."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    vol, osd, gsd, march = config4
    W, H = 3840, 2160
    r.set_volume(vol)
    r.set_shader_data(osd, gsd)
    r.set_march(march)
    for fmt, part in ((1, "auto"), (0, "auto"), (1, "rows")):
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=16, world=8, rank=0, loopback=True, partition=part)
        try:
            pl.run_frames(3)
            if part == "auto":   # the 8-rank default: serpentine band sets, rank 0 compositing + lead rows
                assert pl.partition == "bands" and pl.compositor and pl.serpentine and pl.render_streams == 3
                assert pl.lead_rows > 0 and pl.lead_rows % 16 == 0, pl.lead_rows
            got = pl.frame()
            full = r.render(W, H, fmt)
            torch.cuda.synchronize()
            assert torch.equal(got, full)
        finally:
            pl.close()


def test_region_lists_outlive_destroyed_streams(r, oracle, vol128):
    """Region lists rendered on streams the caller destroys afterwards (the
    native loop's own render streams, gone at close()): later rebuilds -- on
    the GPU and on the host, every render -- must not touch those streams.
    Lists retire with an event recorded on the retiring render's own stream
    when that is the only stream that used them, and with a device sync
    otherwise: never with an event recorded on a remembered stream handle."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 320, 180
    r.set_volume(vol128)
    r.set_march(vr.march_defaults())
    r.set_option("region_interval", 1)
    try:
        for gpu in (1, 0):
            r.set_option("region_gpu", gpu)
            osd, gsd = vr.reference_shader_data(W / H, 3.0, 0.0)
            r.set_shader_data(osd, gsd)
            r.render(W, H, 0)   # lists for the full target on the default stream
            pl = RcclBandPipeline(r, W, H, 0, band_rows=16, world=2, rank=0, loopback=True)
            try:
                pl.run_frames(2)   # rank 0's and rank 1's lists, on the loop's streams
                pl.frame()
            finally:
                pl.close()
            torch.cuda.synchronize()
            for i in range(1, 5):   # spinning: a rebuild every render retires the loop's lists
                osd, gsd = vr.reference_shader_data(W / H, 3.0 + SPIN_DEG * i, 0.0)
                r.set_shader_data(osd, gsd)
                cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
                img = r.render(W, H, 0, step_counter=cnt)
            torch.cuda.synchronize()
            obj, glob = vr.shader_data_arrays(osd, gsd)
            ref, steps = oracle.render(vol128, obj, glob, oracle.from_params(vr.march_defaults()), W, H, 0)
            assert_exact(img.cpu().numpy(), ref)
            assert int(cnt.item()) == steps
    finally:
        r.set_option("region_gpu", 1)
        r.set_option("region_interval", 32)


@pytest.mark.parametrize("cam", [(4.0, 2.0, 2.5), (0.3, -0.2, 0.5), (-4.0, 1.0, 0.0), (3.0, 3.0, 3.0001)])
@pytest.mark.parametrize("layout", [0, 1, 12])
def test_camera_position_off_the_view_eye(r, oracle, vol128, cam, layout):
    """CameraPosition != the View eye: the ray leaves CameraPosition through
    the front-face point the View camera rasterises (frag.glsl:36-38,
    vert.glsl:20).  Exact against the oracle (itself checked against the
    float64 restatement in tests/test_oracle_independent.py), for the auto,
    planar and brick4832 layouts."""
    osd, gsd = vr.reference_shader_data(16 / 9, 20.0, 10.0)
    gsd.camera_position[:] = list(cam)
    r.set_layout_preference(layout)
    try:
        for W, H, band in [(320, 180, {}), (400, 225, dict(band_rows=16, band_stride=3, band_first=1))]:
            img, ref, c, s = render_both(r, oracle, vol128, W, H, osd, gsd, **band)
            assert_exact(img, ref)
            assert c == s
    finally:
        r.set_layout_preference(0)


# ---- the clamp-to-edge proof (vr_api.cpp clamp_is_exact) under adversarial offsets ----

def clamp_is_exact_py(march, glob, dims):
    """Python replica of vr_api.cpp clamp_is_exact / tap_constants: may the
    fast (clamp-to-edge) layouts stand in for MIRRORED_REPEAT this frame?"""
    f32 = np.float32
    slack = (march.max_steps + 16) * 1.2e-7
    for t in range(4):
        for a in range(3):
            off = f32(glob[20 + a * 4 + t]) * f32(march.tap_weight[t])
            S = f32(march.tap_scale[t]) * f32(dims[a])
            T = off * f32(dims[a]) + f32(0.5)
            s, o = float(S), float(T)
            margin = abs(s) * slack + (dims[a] + 2.0) * 2.4e-7 + 1e-6
            lo, hi = min(o, s + o) - margin, max(o, s + o) + margin
            if not (lo >= 0.0 and hi < dims[a] + 1.0):
                return False
    return True


def offset_for_T(T, N, w):
    """A MediaScroll entry that makes the tap's padded offset T = off*N + 0.5 = T (float32)."""
    f32 = np.float32
    v = f32((T - 0.5) / N / w)
    for _ in range(64):   # nudge to the float whose T rounds where asked
        got = float(f32(v) * f32(w) * f32(N) + f32(0.5))
        if got == np.float32(T):
            break
        v = np.nextafter(v, f32(np.inf) if got < T else f32(-np.inf), dtype=np.float32)
    return float(v)


@pytest.mark.parametrize("max_steps", [1, 300])
@pytest.mark.parametrize("edge", ["low", "high"])
def test_wrap_mode_switch_at_the_margin(r, oracle, vol128, max_steps, edge):
    """Tap ranges g within ~1e-6 of 0 and of N+1, on both sides of
    clamp_is_exact's margin: the fast layout runs exactly when the proof
    holds, planar mirrored repeat otherwise, and the frame is exact either
    way -- including offsets where rays entering through a face put taps a
    hair outside [0, N+1), where clamp and mirror really differ."""
    N = 128
    base = vr.march_defaults(max_steps=max_steps)
    slack = (max_steps + 16) * 1.2e-7
    seen = set()
    for t in (1, 3):
        S = float(np.float32(base.tap_scale[t]) * np.float32(N))
        margin = abs(S) * slack + (N + 2.0) * 2.4e-7 + 1e-6
        for delta in (-3e-6, -1e-6, -1e-7, 1e-7, 1e-6, 3e-6, 2e-4):
            # low edge: T just above/below margin; high edge: S + T just below/above N + 1 - margin
            T = margin + delta if edge == "low" else (N + 1.0 - margin) - S + delta
            # rays enter the box through the faces on the edge's side (P = 0 faces
            # for the low edge: the camera rotated to local (-3,-3,3)), so taps at
            # entry points sit right at the edge of the g-range
            osd, gsd = vr.reference_shader_data(16 / 9, 180.0 if edge == "low" else 0.0, 5.0)
            w = float(base.tap_weight[t])
            for a in range(3):
                gsd.media_scroll[a * 4 + t] = offset_for_T(T, N, w)
            obj, glob = vr.shader_data_arrays(osd, gsd)
            exact = clamp_is_exact_py(base, glob, (N, N, N))
            img, ref, c, s = render_both(r, oracle, vol128, 256, 144, osd, gsd, march=base)
            want = "grid_cornerh_clamp" if exact else "grid_planar_mirror"
            assert r.kernel_variant == want, (t, delta, exact)
            assert_exact(img, ref)
            assert c == s
            seen.add(exact)
    assert seen == {True, False}   # both sides of the margin were exercised


@pytest.mark.parametrize("W,H", [(1, 1), (1, 7), (9, 1), (2, 3), (8, 8), (65, 1)])
@pytest.mark.parametrize("layout", [0, 12, 1])
def test_tiny_and_ragged_frames(r, oracle, vol128, W, H, layout):
    """Frames of one pixel, one row, one column and sizes around the 8x8 wave
    tile, through the auto (cornerh), brick4832 and planar paths with the auto
    (regions) schedule: exact, step counts too."""
    r.set_layout_preference(layout)
    try:
        img, ref, c, s = render_both(r, oracle, vol128, W, H)
        assert_exact(img, ref)
        assert c == s
    finally:
        r.set_layout_preference(0)


@pytest.mark.parametrize("W,H,shadow", [(1, 1, 0), (5, 3, 8), (1, 9, 8), (70, 2, 0)])
def test_tiny_frames_procedural(r, oracle, W, H, shadow):
    """The cost-sorted procedural path on frames smaller than one wave."""
    img, ref, c, s, _ = render_proc_both(r, oracle, W, H, vr.march_defaults(), shadow_steps=shadow)
    assert_exact(img, ref)
    assert c == s


@pytest.mark.parametrize("kind,status", [(1, 2), (2, 5)])
def test_exception_never_crosses_the_abi(oracle, vol128, kind, status):
    """Verdict r04 #5: a C++ exception inside an entry point's host path
    (option inject_throw: std::runtime_error / std::bad_alloc thrown inside
    vr_render) comes back as a vr_status -- VR_ERR_HIP / VR_ERR_OOM with the
    message in vr_last_error -- instead of terminating the process; the same
    context then renders exactly again.  The native frame loop passes the
    status through (loopback, 2 ranks) and runs on afterwards."""
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 200, 120
    with vr.Renderer(0) as rr:
        img, ref, cnt, steps = render_both(rr, oracle, vol128, W, H)
        assert_exact(img, ref)
        rr.set_option("inject_throw", kind)
        with pytest.raises(VRError) as e:
            rr.render(W, H, 0)
        assert e.value.status == status, e.value
        assert "vr_render" in str(e.value)
        again = rr.render(W, H, 0)
        torch.cuda.synchronize()
        assert_exact(again.cpu().numpy(), ref)
        pl = RcclBandPipeline(rr, W, H, 0, band_rows=16, world=2, rank=0, loopback=True)
        try:
            pl.run_frames(2)
            rr.set_option("inject_throw", kind)
            with pytest.raises(VRError) as e2:
                pl.run_frames(2)
            assert e2.value.status == status, e2.value
            pl.run_frames(3)
            pl.barrier()
            got = pl.frame()
            torch.cuda.synchronize()
            assert_exact(got.cpu().numpy(), ref)
        finally:
            pl.close()
    with vr.Renderer(0) as r2, pytest.raises(VRError):
        r2.set_option("inject_throw", 3)


def test_launch_cache_hits_and_invalidation(oracle, vol128):
    """The grid launch cache (option launch_cache): repeated renders of an
    unchanged frame on the same stream and target reuse the cached kernel
    arguments (the hit counter moves), and every change that alters the
    launch -- camera, march constants, another target or band set, an option
    -- is seen: each frame equals the oracle's, bit for bit, alternating two
    targets on two streams as the multi-GPU loop does."""
    W, H = 256, 144
    with vr.Renderer(0) as rr:
        rr.set_volume(vol128)
        cams = [vr.reference_shader_data(W / H, a, 0.5 * a) for a in (0.0, 25.0)]
        m2 = vr.march_defaults(max_steps=64)
        assert rr.get_option("launch_cache") == 1
        outs = [rr.alloc_target(W, H, 0), rr.alloc_target(W, H, 0)]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]

        def ref(cam, m, **band):
            obj, glob = vr.shader_data_arrays(*cam)
            return oracle.render(vol128, obj, glob, oracle.from_params(m), W, H, 0, **band)[0]
        for cam, m in ((cams[0], vr.march_defaults()), (cams[1], vr.march_defaults()), (cams[1], m2)):
            rr.set_shader_data(*cam)
            rr.set_march(m)
            h0 = rr.get_option("launch_cache_hits")
            for i in range(6):
                with torch.cuda.stream(streams[i % 2]):
                    rr.render(W, H, 0, out=outs[i % 2])
            torch.cuda.synchronize()
            assert rr.get_option("launch_cache_hits") - h0 >= 4
            want = ref(cam, m)
            for o in outs:
                assert_exact(o.cpu().numpy(), want)
        # a band set on the same buffers, then the whole frame again
        band = dict(band_rows=16, band_stride=3, band_first=1)
        b = rr.render(W, H, 0, **band)
        torch.cuda.synchronize()
        assert_exact(b.cpu().numpy(), ref(cams[1], m2, **band))
        rr.set_option("uniform_skip", 0)
        rr.render(W, H, 0, out=outs[0])
        torch.cuda.synchronize()
        assert_exact(outs[0].cpu().numpy(), ref(cams[1], m2))
        rr.set_option("launch_cache", 0)
        h1 = rr.get_option("launch_cache_hits")
        rr.render(W, H, 0, out=outs[1])
        rr.render(W, H, 0, out=outs[1])
        torch.cuda.synchronize()
        assert rr.get_option("launch_cache_hits") == h1
        assert_exact(outs[1].cpu().numpy(), ref(cams[1], m2))


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_bands_in_place_and_partial_assembly(oracle, vol128, fmt):
    """VR_TARGET_BANDS_IN_PLACE (vr.h): band sets rendered at their own frame
    rows of a whole-frame buffer -- every rank's set in turn -- give the plain
    whole-frame render bit for bit, and a set leaves the other rows as they
    were (NaN / 0xAB prefill).  vr_assemble_frame_ranks(first_rank = 1) fills
    the other ranks' rows from grey gather slots and leaves rank 0's rows
    untouched (the multi-GPU loop's rank 0, vr_shard.cpp)."""
    import ctypes
    from volumetricrenderer_amd import _lib
    W, H, N, B = 301, 170, 3, 16
    with vr.Renderer(0) as rr:
        rr.set_volume(vol128)
        rr.set_shader_data(*vr.reference_shader_data(W / H, 20.0, -10.0))
        rr.set_march(vr.march_defaults())
        full = rr.render(W, H, fmt)
        frame = rr.alloc_target(W, H, fmt)
        if frame.dtype == torch.float32:
            frame.fill_(float("nan"))
        else:
            frame.fill_(0xAB)
        pitch = frame.stride(0) * frame.element_size()

        def in_place(first):
            t = _lib.Target(width=W, height=H, format=fmt | _lib.TARGET_BANDS_IN_PLACE, band_rows=B, band_stride=N,
                            band_first=first, pixels=frame.data_ptr(), row_pitch=pitch, step_counter=None)
            _lib.call("vr_render", rr._ctx, ctypes.byref(t), None)
        in_place(1)
        torch.cuda.synchronize()
        got, want = frame.cpu().numpy(), full.cpu().numpy()
        rows1 = [y for y in range(H) if (y // B) % N == 1]
        other = [y for y in range(H) if (y // B) % N != 1]
        assert np.array_equal(got[rows1], want[rows1])
        if fmt == 0:
            assert np.isnan(got[other]).all()
        else:
            assert (got[other] == 0xAB).all()
        in_place(0)
        in_place(2)
        torch.cuda.synchronize()
        assert np.array_equal(frame.cpu().numpy(), want)
        # rank 0 in place, ranks 1..N-1 as grey sets in gather slots
        g = {0: 5, 1: 3, 2: 4}[fmt]
        rpr = vr.band_rows_packed(H, B, N, 0)
        gathered = torch.zeros((N, rpr) + tuple(rr.alloc_target(W, 1, g).shape[1:]), dtype=rr.alloc_target(W, 1, g).dtype,
                               device="cuda")
        for r in range(1, N):
            rr.render(W, H, g, out=gathered[r][: vr.band_rows_packed(H, B, N, r)], band_rows=B, band_stride=N,
                      band_first=r)
        if frame.dtype == torch.float32:
            frame.fill_(float("nan"))
        else:
            frame.fill_(0xAB)
        in_place(0)
        _lib.call("vr_assemble_frame_ranks", rr._ctx, ctypes.c_void_p(gathered.data_ptr()), g, rpr, N, 1, W, H, B, fmt,
                  ctypes.c_void_p(frame.data_ptr()), None)
        torch.cuda.synchronize()
        assert np.array_equal(frame.cpu().numpy(), want)


@pytest.mark.parametrize("fmt", [0, 1, 3])
def test_row_ranges_match_the_frame(oracle, vol128, fmt):
    """VR_TARGET_ROW_RANGE (vr.h): contiguous row ranges -- the multi-GPU
    loop's balanced partition (vr_shard_balance_rows) -- packed or in place,
    equal the whole frame's rows bit for bit; ranges run past the frame's
    last row without writing there, and a range's first row must be a
    multiple of 8.  vr_row_partition's ranges tile the frame, its boundaries
    are multiples of 8, and the executed steps of the ranges are balanced
    (each within 35 % of the mean: 8-row granules of a 203-row frame)."""
    import ctypes
    from volumetricrenderer_amd import _lib
    W, H = 333, 203
    with vr.Renderer(0) as rr:
        rr.set_volume(vol128)
        rr.set_shader_data(*vr.reference_shader_data(W / H, 25.0, 15.0))
        rr.set_march(vr.march_defaults())
        full = rr.render(W, H, fmt)
        sc = torch.zeros(1, dtype=torch.int64, device="cuda")
        rr.render(W, H, fmt, step_counter=sc)
        want = full.cpu().numpy()
        for first, n in ((0, 8), (0, 64), (40, 57), (96, 107), (200, 64), (8, 1)):
            got = rr.render_rows(W, H, fmt, first, n)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), want[first:first + n]), (first, n)
        # in place: every range of a partition into a prefilled frame
        frame = rr.alloc_target(W, H, fmt)
        frame.fill_(float("nan") if frame.dtype == torch.float32 else 0xAB)
        rb = rr.row_partition(W, H, 5)
        assert rb[0] == 0 and rb[-1] == H and all(b % 8 == 0 for b in rb[1:-1])
        assert all(a <= b for a, b in zip(rb, rb[1:]))
        # the strip work it splits (vr_row_work): boundary k sits at the strip
        # edge nearest the k/5 quantile of the prefix sums
        sw = np.array(rr.row_work(W, H))
        assert sw.shape == ((H + 7) // 8,) and (sw > 0).all()
        pre = np.concatenate([[0.0], np.cumsum(sw)])
        for k in range(1, 5):
            e = int(np.argmin(np.abs(pre - pre[-1] * k / 5)))
            assert abs(rb[k] // 8 - e) <= 1, (k, rb, e)
        with pytest.raises(vr.VRError):   # nstrips must be ceil(H / 8)
            _lib.call("vr_row_work", rr._ctx, W, H, (ctypes.c_double * 3)(), 3)
        for k in range(5):
            if rb[k + 1] > rb[k]:
                rr.render_rows(W, H, fmt, rb[k], rb[k + 1] - rb[k], out=frame, in_place=True)
        torch.cuda.synchronize()
        assert np.array_equal(frame.cpu().numpy(), want)
        # the ranges' executed steps: balanced
        steps = []
        for k in range(5):
            c = torch.zeros(1, dtype=torch.int64, device="cuda")
            out = rr.alloc_target(W, max(1, rb[k + 1] - rb[k]), fmt)
            t = _lib.Target(width=W, height=H, format=fmt | _lib.TARGET_ROW_RANGE, band_rows=max(1, rb[k + 1] - rb[k]),
                            band_stride=1, band_first=rb[k], pixels=out.data_ptr(),
                            row_pitch=out.stride(0) * out.element_size(), step_counter=c.data_ptr())
            _lib.call("vr_render", rr._ctx, ctypes.byref(t), None)
            torch.cuda.synchronize()
            steps.append(int(c.item()))
        assert sum(steps) == int(sc.item())
        mean = sum(steps) / 5
        assert max(abs(s - mean) for s in steps) <= 0.35 * mean, (rb, steps)
        for bad in ((4, 16, 1), (0, 16, 2), (0, 0, 1)):   # first not a multiple of 8, stride, no rows
            t = _lib.Target(width=W, height=H, format=fmt | _lib.TARGET_ROW_RANGE, band_rows=bad[1],
                            band_stride=bad[2], band_first=bad[0], pixels=full.data_ptr(),
                            row_pitch=full.stride(0) * full.element_size(), step_counter=None)
            with pytest.raises(vr.VRError):
                _lib.call("vr_render", rr._ctx, ctypes.byref(t), None)
        with pytest.raises(vr.VRError):
            rr.row_partition(W, H, 0)
