"""Sprites through the Trident::Renderer shim: GatherSpriteDraws / DrawSprites
(Trident/src/Renderer/Renderer.cpp:2996-3089) draw every visible SpriteComponent after the meshes in the same
pass, with the Default pipeline's state, over the quad of BuildSpriteGeometry (:2853-2890, indices
{0, 2, 1, 0, 3, 2}) and the only non-default push constants of the reference: tint, UV scale / offset,
tiling, the material-override flag, the sort offset and the texture slot (:3065-3083). `.trident` files
keep Sprite lines (Scene.cpp:343-367, :549-779).

CPU tests check the submitted geometry and draw list; the GPU test renders tinted, UV-scaled, textured
sprites over meshes and compares with the oracle on the shim's own inputs.
"""
import numpy as np
import pytest

from test_host_shim import app_mod, assert_shim_parity  # noqa: F401  (fixture)


def sprite_app(app_mod):  # noqa: F811
    a = app_mod.TridentApp()
    a.set_camera("editor", (0.0, 0.5, 5.0))
    a.set_viewport(1, 320, 240)
    a.add_mesh_entity("cube", position=(0.0, -0.8, -1.0), rotation=(15.0, 30.0, 0.0), scale=(1.5, 1.5, 1.5))
    # facing the camera: the sprite quad faces -Z, so it is turned 180 degrees about Y (front-facing)
    s1 = a.add_sprite_entity(position=(-1.1, 0.6, 0.5), rotation=(0.0, 180.0, 0.0), scale=(1.4, 1.0, 1.0),
                             tint=(1.0, 0.6, 0.4, 0.8), uv_scale=(2.0, 1.5), uv_offset=(0.25, -0.1), tiling=1.5)
    s2 = a.add_sprite_entity(position=(1.0, 0.4, 0.0), rotation=(0.0, 200.0, 10.0), scale=(1.2, 1.2, 1.0),
                             tint=(0.5, 0.9, 1.0, 1.0))
    # not turned: back-facing from this camera, culled like the reference's (cull BACK on the quad)
    s3 = a.add_sprite_entity(position=(0.0, 1.2, 0.0), scale=(3.0, 3.0, 1.0))
    return a, (s1, s2, s3)


def test_sprite_draws_follow_the_meshes(app_mod):  # noqa: F811
    a, (s1, s2, s3) = sprite_app(app_mod)
    ubo, draws = a.frame_inputs(1)
    vb, ib, ranges = a.geometry()
    assert len(draws) == 4 and draws[0].mesh_index == 0  # the cube, then the three sprites in entity order
    sprite_mesh = draws[1].mesh_index
    assert sprite_mesh == len(ranges) - 1 and all(d.mesh_index == sprite_mesh for d in draws[1:])
    first, count, base, mat = ranges[sprite_mesh]
    assert count == 6 and mat == -1
    assert ib[first:first + 6].tolist() == [0, 2, 1, 0, 3, 2]
    quad = vb[base:base + 4]
    assert quad["position"].tolist() == [[-0.5, -0.5, 0], [0.5, -0.5, 0], [0.5, 0.5, 0], [-0.5, 0.5, 0]]
    assert (quad["normal"] == [0, 0, -1]).all() and (quad["color"] == 1).all()
    assert quad["texcoord"].tolist() == [[0, 0], [1, 0], [1, 1], [0, 1]]
    pc = draws[1].pc
    assert tuple(pc.tint) == pytest.approx((1.0, 0.6, 0.4, 0.8))
    assert tuple(pc.texture_scale) == (2.0, 1.5) and tuple(pc.texture_offset) == pytest.approx((0.25, -0.1))
    assert pc.tiling_factor == 1.5 and pc.material_index == -1 and pc.texture_slot == 0
    assert pc.bone_offset == 0 and pc.bone_count == 0
    assert tuple(draws[3].pc.tint) == (1, 1, 1, 1) and tuple(draws[3].pc.texture_scale) == (1, 1)
    a.set_sprite_visible(s2, False)  # invisible sprites are skipped (Renderer.cpp:3016-3019)
    _, draws = a.frame_inputs(1)
    assert len(draws) == 3
    a.close()


def test_sprite_texture_component_slot(app_mod):  # noqa: F811
    a, (s1, s2, s3) = sprite_app(app_mod)
    tex = np.full((4, 4, 4), 200, np.uint8)
    a.upload_texture("sprite.png", tex)
    a.set_entity_texture(s2, "sprite.png")
    _, draws = a.frame_inputs(1)
    assert [d.pc.texture_slot for d in draws] == [0, 0, 1, 0]
    a.close()


def test_sprite_scene_round_trip(app_mod, tmp_path):  # noqa: F811
    a, (s1, s2, s3) = sprite_app(app_mod)
    a.set_sprite_visible(s3, False)
    p = tmp_path / "sprites.trident"
    a.save_scene(p)
    text = p.read_text()
    assert "Sprite Texture=\"\" Tint=1,0.6,0.4,0.8 UVScale=2,1.5 UVOffset=0.25,-0.1 Tiling=1.5 Visible=true" in text
    assert "UseMaterialOverride=false AtlasTiles=1,1 AtlasIndex=0 AnimationSpeed=0 SortOffset=0" in text
    b = app_mod.TridentApp()
    b.set_camera("editor", (0.0, 0.5, 5.0))
    b.set_viewport(1, 320, 240)
    assert b.load_scene(p) == 4
    for e in (1, 2, 3):
        ga, gb = a.entity_sprite(e), b.entity_sprite(e)
        for k in ga:
            assert np.allclose(ga[k], gb[k], atol=1e-6), (e, k)
    _, da = a.frame_inputs(1)
    _, db = b.frame_inputs(1)
    assert [bytes(memoryview(d.pc))[64:] for d in db] == [bytes(memoryview(d.pc))[64:] for d in da]
    a.close()
    b.close()


@pytest.mark.gpu
def test_gpu_sprites_over_meshes(app_mod, oracle):  # noqa: F811
    """Tinted, UV-scaled / offset, tiled sprites (one textured through a TextureComponent, one with alpha
    tint, one back-facing and culled) over a cube: depth bit-exact, colour within 1 LSB of the oracle."""
    a, (s1, s2, s3) = sprite_app(app_mod)
    yy, xx = np.mgrid[0:8, 0:8]
    checker = np.where(((xx + yy) % 2)[..., None] == 0, 220, 40).astype(np.uint8).repeat(4, -1)
    checker[..., 3] = 255
    a.upload_texture("checker.png", checker)
    a.set_entity_texture(s1, "checker.png")
    a.add_light("point", position=(0.0, 1.5, 2.5), color=(1.0, 0.9, 0.8), intensity=6.0, range=8.0)
    a.draw_frame()
    a.draw_frame()
    assert_shim_parity(a, oracle, 1, 320, 240, textures=[(1, checker)], min_covered=8000)
    rgba_on, _ = a.read_pixels(1, 320, 240)
    for s in (s1, s2, s3):
        a.set_sprite_visible(s, False)
    a.draw_frame()
    rgba_off, _ = a.read_pixels(1, 320, 240)
    assert int((np.abs(rgba_on.astype(np.int16) - rgba_off.astype(np.int16)).max(-1) > 8).sum()) > 3000  # visible
    assert_shim_parity(a, oracle, 1, 320, 240, textures=[(1, checker)], min_covered=2000)
    a.close()
