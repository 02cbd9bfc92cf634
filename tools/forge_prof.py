"""Forge's editor frame through the engine API alone (bench.forge_frame), for a rocprofv3 kernel trace:
python tools/forge_prof.py [4k|panels] [frames_in_flight]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d-renderer_amd", "python"))

import bench  # noqa: E402

layout = bench.FORGE_4K if (sys.argv[1:2] or ["4k"])[0] == "4k" else bench.FORGE_PANELS
fif = int(sys.argv[2]) if len(sys.argv) > 2 else 3
print(json.dumps(bench.forge_frame(layout, frames_in_flight=fif)))
