# round 6: one bench line per BASELINE.json config and SURVEY 8f mode on the final build
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/sweep
sweep && echo sweep_done
