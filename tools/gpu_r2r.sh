set -o pipefail
mkdir -p gpurun_out/r2r
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w -o /tmp/ll tools/launch_latency.hip &&
timeout -k 5 60 /tmp/ll > gpurun_out/r2r/launch.json &&
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_sstrace.so timeout -k 10 200 python3 tools/single_shot_trace.py > gpurun_out/r2r/trace.json 2> gpurun_out/r2r/ss.err
