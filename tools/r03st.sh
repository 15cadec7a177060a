# End of round 3: the config-5 stream demo (300 rendered 1080p frames, GPU front-end, 30-KF sliding-window BA)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python pan-tilt-zoom-slam_amd/demo_stream.py --frames 300 > gpurun_out/r03st_demo_stream.json 2> gpurun_out/r03st_demo_stream.err || { echo DEMOFAIL; tail -20 gpurun_out/r03st_demo_stream.err; exit 1; }
tail -c 1500 gpurun_out/r03st_demo_stream.json
