"""The reference's HDR output convention: main_taichi.py:120-123 saves the
radiance SUMS `pixels.to_numpy()` as hdr.npy and the per-pixel sample counts `samples.to_numpy()` as
spp.npy; the reference's offline tone_map.py:5-9 reads exactly that pair (NaN -> 0, then
sqrt(hdr / spp[0, 0])).  `python -m pyrenderer_amd --hdr DIR` writes the pair with
tone_map.save_hdr; here the reference's formula, applied to the loaded files, must reproduce
tone_map.finish of the mean image (render()'s sums / spp) bit for bit."""
import numpy as np

from pyrenderer_amd.tone_map import finish, finish_hdr, save_hdr


def test_hdr_pair_reproduces_finish_of_the_mean(tmp_path):
    rng = np.random.default_rng(3)
    spp = 37
    sums = (rng.random((48, 32, 3), dtype=np.float32) * np.float32(spp * 2.5)).astype(np.float32)
    sums[5, 7, 1] = np.nan                               # a non-finite sample sum (the reference zeroes it)
    hdr_p, spp_p = save_hdr(str(tmp_path / "out"), sums, spp)
    hdr_mat, spp_mat = np.load(hdr_p), np.load(spp_p)
    assert hdr_mat.dtype == np.float32 and hdr_mat.shape == (48, 32, 3)
    assert spp_mat.dtype == np.float32 and spp_mat.shape == (48, 32) and (spp_mat == spp).all()
    # tone_map.py:5-9, as the reference runs it on the loaded pair
    ref = hdr_mat.copy()
    ref[np.isnan(ref)] = 0
    ldr1 = np.sqrt(ref / spp_mat[0, 0])
    # the build's finish() of the mean render() returns (sums / spp), NaN pixel zeroed the same way
    clean = np.where(np.isnan(sums), np.float32(0), sums)
    mean = clean / np.float32(spp)
    np.testing.assert_array_equal(ldr1, finish(mean))
    np.testing.assert_array_equal(finish_hdr(hdr_mat, spp_mat), ldr1)
    assert np.array_equal(hdr_mat[~np.isnan(hdr_mat)], sums[~np.isnan(sums)])   # the sums themselves


def test_cli_rejects_an_npy_file_for_the_hdr_directory(capsys):
    """`--hdr out.npy` (the pre-round-5 file form) is refused instead of silently creating a
    directory named out.npy."""
    import pytest
    from pyrenderer_amd.main import parse
    assert parse(["--hdr", "outdir"]).hdr == "outdir"
    with pytest.raises(SystemExit) as e:
        parse(["--hdr", "out.npy"])
    assert e.value.code == 2 and "directory" in capsys.readouterr().err
