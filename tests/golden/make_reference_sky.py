"""Crop the reference's own rendered frame into the sky-pass fixtures (run in the build container, where
/root/reference exists; the GPU box only reads the committed PNGs).

Source: `Screenshots/Screenshot1.png` (2559x1439 RGBA) of the reference checkout: a Trident-Forge window
showing a skybox-only scene (hierarchy: one Camera entity, no meshes) in its two viewports, rendered by
the reference's Vulkan path (Skybox.vert:30-41, Skybox.frag:28-35, the PNG cubemap found by
Renderer.cpp:3830-3927) and displayed 1:1 by ImGui.

- Scene viewport: rows 80..1157, cols 8..999   (992x1078), editor camera.
- Game viewport:  rows 80..1157, cols 1018..2081 (1064x1078), runtime camera; the "FPS: ..." label the
  Game panel draws over the image (GameViewportPanel.cpp) covers rows 12..30, cols 12..153 of the crop, so
  the test masks rows 8..35, cols 8..160 there.

The crops are stored losslessly as RGB PNG (tests/golden/reference_sky_{scene,game}.png). They are reference
OUTPUT used as expected values (test data), not reference source.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/Screenshots/Screenshot1.png"

# (row0, row1, col0, col1), half-open
CROPS = {"scene": (80, 1158, 8, 1000), "game": (80, 1158, 1018, 2082)}
GAME_LABEL_MASK = (8, 36, 8, 161)  # rows, cols inside the game crop


def main(src=SRC):
    from PIL import Image

    a = np.asarray(Image.open(src).convert("RGBA"))
    assert a.shape == (1439, 2559, 4), a.shape
    for name, (y0, y1, x0, x1) in CROPS.items():
        crop = np.ascontiguousarray(a[y0:y1, x0:x1, :3])
        # the crop must be exactly the viewport image: the ImGui panel background (15,15,15) lies on all four
        # sides, one pixel outside it
        for edge in (a[y0 - 1, x0:x1, :3], a[y1, x0:x1, :3], a[y0:y1, x0 - 1, :3], a[y0:y1, x1, :3]):
            assert np.all(edge == 15), name
        out = os.path.join(HERE, f"reference_sky_{name}.png")
        Image.fromarray(crop, "RGB").save(out, optimize=True)
        print(out, crop.shape)


if __name__ == "__main__":
    main(*sys.argv[1:])
