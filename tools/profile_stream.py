#!/usr/bin/env python3
"""Host profile of the config-5 stream (demo_stream.py) under cProfile: where a keyframe BA call spends its wall time
on the Python side.  Writes the pstats tables (cumulative and own time, top 60) to the given file; the demo's JSON
line goes to stdout as usual.

  python tools/profile_stream.py OUT.txt [demo_stream args ...]
"""
import cProfile
import io
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pan-tilt-zoom-slam_amd"))


def main():
    out = sys.argv[1]
    sys.argv = ["demo_stream.py"] + sys.argv[2:]
    import demo_stream
    prof = cProfile.Profile()
    prof.enable()
    demo_stream.main()
    prof.disable()
    buf = io.StringIO()
    st = pstats.Stats(prof, stream=buf)
    st.sort_stats("cumulative").print_stats(60)
    st.sort_stats("tottime").print_stats(60)
    st.print_callers("landmark_index|_same_image|array_equal|_materialise|hasattr")
    with open(out, "w") as f:
        f.write(buf.getvalue())


if __name__ == "__main__":
    main()
