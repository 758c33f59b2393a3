set -o pipefail
for a in FrodoKEM-640-SHAKE FrodoKEM-976-SHAKE FrodoKEM-640-AES; do
  timeout -k 10 400 bash tools/profile.sh r2_$a --alg $a &&
  timeout -k 10 200 bash tools/pmc_mfma.sh r2_$a --alg $a || exit 1
done
