"""The Python mirror's host-side pieces (no GPU): search.bresenham against the reference's pixel
lists (F3), and the map loader of main.py:37-42 (PNG -> Image.convert('1') -> bool imarray) on the
reference's maps (map1/map2 as stored in tests/golden/maps.npz, written back out as the RGB 0/255
PNGs the reference ships)."""
import builtins

import numpy as np
import pytest

from conftest import golden
import pkgload

pkgload.load()
from theta_rrt_amd import config, search  # noqa: E402


def test_search_bresenham_golden():
    f = golden("f3_bres.npz")
    seg, off, pix = f["seg"], f["off"], f["pix"]
    for i, (a, b, c, d) in enumerate(seg.tolist()):
        assert search.bresenham((a, b), (c, d)) == [tuple(p) for p in pix[off[i]:off[i + 1]].tolist()]


@pytest.mark.parametrize("name", ["map1", "map2"])
def test_load_map_roundtrip(tmp_path, maps, name):
    from PIL import Image
    m = maps[name]
    rgb = np.repeat((m.astype(np.uint8) * 255)[:, :, None], 3, axis=2)     # as map1.png / map2.png
    path = str(tmp_path / (name + ".png"))
    Image.fromarray(rgb, "RGB").save(path)
    got = config.load_map(path)
    assert got.dtype == bool and got.shape == m.shape
    assert np.array_equal(got, m)
    assert builtins.imarray is got
    # gray and 1-bit inputs decode to the same occupancy
    Image.fromarray(m.astype(np.uint8) * 255, "L").save(path)
    assert np.array_equal(config.load_map(path), m)
    Image.fromarray(m).save(path)
    assert np.array_equal(config.load_map(path), m)


def test_grid_changed_bumps_the_upload_key():
    v = config._grid_key[1]
    config.grid_changed()
    assert config._grid_key[1] == v + 1


def test_config_engine_uploads_again_after_a_direct_set_grid(monkeypatch):
    """config.engine() keys the uploaded map by array identity; a set_grid made on the process
    engine directly in between (another map) must not pass for it."""
    import builtins
    from theta_rrt_amd import _native, config

    class FakeEngine:
        def __init__(self):
            self.uploads, self.grid_serial = [], 0

        def set_params(self, p):
            pass

        def set_grid(self, a):
            self.uploads.append(np.array(a, copy=True))
            self.grid_serial += 1
    fake = FakeEngine()
    monkeypatch.setattr(_native, "engine", lambda: fake)
    monkeypatch.setattr(config, "_grid_key", [None, 0, None, -1])
    config.ensure_defaults()
    a = np.ones((6, 6), bool)
    monkeypatch.setattr(builtins, "imarray", a, raising=False)
    config.engine()
    config.engine()
    assert len(fake.uploads) == 1                     # same array, unchanged: one upload
    fake.set_grid(np.zeros((4, 4), bool))             # somebody uses the engine with another map
    config.engine()
    assert len(fake.uploads) == 3 and fake.uploads[-1].shape == (6, 6)
