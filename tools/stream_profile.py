"""Where a tracked frame's time goes in the config-5 loop with the GPU front-end: cProfile of run_stream over
rendered 1080p frames (frames rendered before profiling)."""
import contextlib
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
import synthetic  # noqa: E402
from demo_stream import run_stream  # noqa: E402
from ptz_slam import PtzSlam  # noqa: E402
from scene_map import Map  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
scene = synthetic.StreamScene(n, seed=0, pan_lo=-10, pan_hi=10)
src = synthetic.RenderedStream(scene)
for i in range(n):
    src.image(i)
slam = PtzSlam()
slam.keyframe_map = Map("sift", max_ba_frame=30)
pr = cProfile.Profile()
with contextlib.redirect_stdout(io.StringIO()):
    pr.enable()
    rec = run_stream(slam, src, n, scene.camera(0), keyframe_every=5)
    pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumtime").print_stats(45)
