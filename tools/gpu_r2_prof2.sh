# rocprof trace + FETCH/WRITE passes for the lines whose traffic was missing or stale
set -o pipefail
bash tools/profile.sh hqc128_r2 --alg HQC-128 > gpurun_out/prof2.log 2>&1 &&
bash tools/profile.sh frodo976aes_r2 --alg FrodoKEM-976-AES >> gpurun_out/prof2.log 2>&1 &&
bash tools/profile.sh frodo1344aes_r2 --alg FrodoKEM-1344-AES >> gpurun_out/prof2.log 2>&1 &&
bash tools/profile.sh frodo1344_r2 --alg FrodoKEM-1344-SHAKE >> gpurun_out/prof2.log 2>&1 &&
bash tools/profile.sh mlkem1024_r2 --alg ML-KEM-1024 >> gpurun_out/prof2.log 2>&1
