#!/bin/bash
# One parametrised runner for every GPU-box step (replaces the round-2 one-off gpu_r2*.sh,
# profile.sh, pmc_sq.sh, pmc_mfma.sh scripts).  Source it inside one gpurun call and chain
# steps with && so the first failure ends the call:
#
#   gpurun -- 'source tools/gpu.sh && out r3a && suite tests/test_gpu_ordering.py &&
#              ab 3 default tree:abtrees/r1head -- --steps 20 --warmup 5 && prof mlkem768'
#
#   out <dir>                 results go to gpurun_out/<dir>/ (merged back by gpurun)
#   suite [pytest targets]    pytest -m gpu (one process), log in suite.log
#   smoke                     __graft_entry__.smoke()
#   bench <tag> [args]        one bench.py line -> <tag>.json (stderr <tag>.err)
#   ab <rounds> <tag>... -- [args]
#                             interleaved A/B (A B A B ...) of library variants inside this one
#                             call, one JSON summary line per run -> ab_<tags>.jsonl.  Tags:
#                             default (in-tree libqrkem.so), <name> (qrkem/variants/libqrkem_<name>.so
#                             from tools/build_variant.sh), tree:<dir> (<dir>/bench.py with that
#                             tree's own package and library, e.g. an older commit's build)
#   prof <tag> [args]         rocprofv3 --kernel-trace --stats, then FETCH_SIZE and WRITE_SIZE in
#                             separate --pmc passes (TCC slots), never combined with tracing
#   sq <tag> [args]           two SQ counter passes (instruction mix, stalls, LDS)
#   mfma <tag> [args]         int8 MFMA counter pass
#   probe <name> <hip> [flags]  build tools/<hip> with hipcc and run it -> <name>.txt
#   pmcbin <name> <binary> <counter...>   one --pmc pass over a prebuilt probe binary
#   run <tag> <command...>    any other GPU command -> <tag>.txt
#   sweep                     one bench line per BASELINE config and SURVEY 8f mode
# Every GPU step runs under its own timeout; a failing step returns non-zero.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/misc
out() { O=$R/gpurun_out/$1; mkdir -p "$O"; }

suite() {
  timeout -k 10 ${SUITE_TIMEOUT:-900} python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    "${@:-tests}" > "$O/suite.log" 2>&1
  local rc=$?
  tail -3 "$O/suite.log"
  return $rc
}

smoke() {
  timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1
}

bench() {
  local tag=$1; shift
  timeout -k 10 ${BENCH_TIMEOUT:-400} python3 "$R/bench.py" "$@" > "$O/$tag.json" 2> "$O/$tag.err"
  local rc=$?
  echo "bench $tag rc=$rc"
  return $rc
}

_ab_one() {  # tag, bench args...
  local t=$1; shift
  local lib= py=$R/bench.py
  case "$t" in
    default) lib=$R/quantum-resistant-p2p_amd/qrkem/libqrkem.so ;;
    tree:*) py=$R/${t#tree:}/bench.py; lib=$R/${t#tree:}/quantum-resistant-p2p_amd/qrkem/libqrkem.so ;;
    *) lib=$R/quantum-resistant-p2p_amd/qrkem/variants/libqrkem_$t.so ;;
  esac
  local o
  o=$(QRKEM_LIBRARY=$lib timeout -k 10 ${AB_TIMEOUT:-240} python3 "$py" --no-cpu "$@" 2>>"$O/ab.err") || return 1
  python3 -c "
import json,sys
d=json.loads(sys.argv[2])
k=d.get('kernels') or {}
tr=d.get('kernels_timed_region') or d.get('kernels_timed_region_forked') or {}
print(json.dumps({'tag':sys.argv[1],'value':d['value'],'ms_per_step':d['ms_per_step'],
  'kernels_serial':{n:round(v['avg_ms'],4) for n,v in k.items()},
  'kernels_timed_region':{n:round(v['avg_ms'],4) for n,v in tr.items()}}))" "$t" "$o"
}

ab() {
  local rounds=$1; shift
  local tags=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do tags+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  local f=$O/ab_$(echo "${tags[*]}" | sed 's#[ /:]#_#g').jsonl
  for r in $(seq 1 "$rounds"); do
    for t in "${tags[@]}"; do
      _ab_one "$t" "$@" >> "$f" || { echo "ab $t failed"; return 1; }
    done
  done
  echo "ab done -> $f"
}

# abx <rounds> <label>=<tag>[,<bench arg>...] ... -- [common args]: interleaved A/B like ab, where
# each variant is a library tag (as in ab) plus its own bench arguments (comma-separated), e.g.
#   abx 3 s0=default s1=default,--streams,1 r3=tree:abtrees/r3head -- --steps 20
abx() {
  local rounds=$1; shift
  local vs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do vs+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  local f=$O/abx.jsonl
  for r in $(seq 1 "$rounds"); do
    for v in "${vs[@]}"; do
      local label=${v%%=*} spec=${v#*=}
      local tag=${spec%%,*} extra=
      [ "$spec" != "$tag" ] && extra=${spec#*,}
      _ab_one "$tag" $(echo "$extra" | tr ',' ' ') "$@" | sed "s/^{\"tag\": \"[^\"]*\"/{\"tag\": \"$label\"/" >> "$f" ||
        { echo "abx $label failed"; return 1; }
    done
  done
  echo "abx done -> $f"
}

prof() {
  local tag=$1; shift
  local d=$O/prof_$tag
  mkdir -p "$d"
  ( export TMPDIR=/tmp; cd /tmp &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -o run -- \
      python3 "$R/bench.py" --steps ${PROF_STEPS:-5} --warmup ${PROF_WARMUP:-1} --no-cpu "$@" \
      > "$d/bench_trace.json" 2> "$d/trace.err" &&
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$d/bench_fetch.json" 2> "$d/fetch.err" &&
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d/write" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$d/bench_write.json" 2> "$d/write.err" )
  local rc=$?
  echo "prof $tag rc=$rc"
  return $rc
}

sq() {
  local tag=$1; shift
  local d=$O/sq_$tag
  mkdir -p "$d"
  ( export TMPDIR=/tmp; cd /tmp &&
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$d/a" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$d/bench_a.json" 2> "$d/a.err" &&
    timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS \
      SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$d/b" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$d/bench_b.json" 2> "$d/b.err" )
  local rc=$?
  echo "sq $tag rc=$rc"
  return $rc
}

mfma() {
  local tag=$1; shift
  local d=$O/mfma_$tag
  mkdir -p "$d"
  ( export TMPDIR=/tmp; cd /tmp &&
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$d/m" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$d/bench_m.json" 2> "$d/m.err" )
  local rc=$?
  echo "mfma $tag rc=$rc"
  return $rc
}

probe() {
  local name=$1 src=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w "$@" -o "/tmp/probe_$name" "$R/tools/$src" || return 1
  timeout -k 5 ${PROBE_TIMEOUT:-120} "/tmp/probe_$name" > "$O/$name.txt" 2>&1
  local rc=$?
  echo "probe $name rc=$rc"
  return $rc
}

# pmcbin <name> <binary> <counter...>: one --pmc pass over a prebuilt probe binary (e.g.
# tools/fetch_calib), stdout -> <name>.out, counters under <name>/
pmcbin() {
  local name=$1 bin=$2; shift 2
  ( export TMPDIR=/tmp; cd /tmp &&
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o run -- "$R/$bin" > "$O/$name.out" 2> "$O/$name.err" )
  local rc=$?
  echo "pmcbin $name rc=$rc"
  return $rc
}

# run <tag> <command...>: any GPU command under a 300 s limit, stdout+stderr -> <tag>.txt
run() {
  local tag=$1; shift
  timeout -k 10 ${RUN_TIMEOUT:-300} "$@" > "$O/$tag.txt" 2>&1
  local rc=$?
  echo "run $tag rc=$rc"
  return $rc
}

# sweep: one bench line (CPU baseline included) for every BASELINE.json config and SURVEY 8f mode
sweep() {
  bench mlkem768 && bench mlkem512 --alg ML-KEM-512 && bench mlkem1024 --alg ML-KEM-1024 &&
  bench mlkem1024_tampered --alg ML-KEM-1024 --mode decaps-tampered &&
  bench mlkem768_2p24 --global-log2-batch 24 --steps 3 --warmup 1 &&
  bench frodo640 --alg FrodoKEM-640-SHAKE && bench frodo976 --alg FrodoKEM-976-SHAKE &&
  bench frodo1344 --alg FrodoKEM-1344-SHAKE --steps 3 --warmup 1 &&
  bench frodo640aes --alg FrodoKEM-640-AES && bench frodo976aes --alg FrodoKEM-976-AES &&
  bench frodo1344aes --alg FrodoKEM-1344-AES --steps 3 --warmup 1 &&
  bench hqc128 --alg HQC-128 && bench hqc192 --alg HQC-192 && bench hqc256 --alg HQC-256 &&
  bench hqc128_tampered --alg HQC-128 --mode decaps-tampered &&
  bench handshake_mlkem768 --mode handshake &&
  bench handshake_frodo976aes --alg FrodoKEM-976-AES --mode handshake --steps 3 --warmup 1 &&
  bench handshake_hqc128 --alg HQC-128 --mode handshake &&
  bench wire_mlkem768 --mode wire
}
