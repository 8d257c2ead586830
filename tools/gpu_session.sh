#!/bin/bash
# One GPU-box call made of named steps, each under its own time limit and
# chained so the first failure ends the call (no GPU step after a fault).
#
#   gpurun --timeout 1200 -- bash tools/gpu_session.sh TAG STEP [STEP ...]
#
# Steps (output under gpurun_out/TAG/):
#   tests              the -m gpu suite (python -u, per-test timeout)
#   parity             tests/test_gpu_parity.py only
#   bench              the default bench.py line (config B, 20 steps, e2e, cpu baseline)
#   bench:CFG[:KCFG]   bench.py --config CFG (B|C|D|E|H), 3 steps, optional forced kernel cfg
#   benchn:CFG:N[:KCFG] the same with N ZMWs per GPU
#   ab:CFG:KCFG,...[:LIB,...]  3 interleaved rounds of bench --config CFG over kernel cfgs x libraries
#   abx:LINE:LIB,...   3 interleaved rounds of bench lines (B|C|D|E16k) over libraries
#   e2e:N[:KCFG]       bench.py's end-to-end line (config E, ccsx_gpu_run) on N ZMWs per GPU
#   kt:CFG             rocprofv3 kernel-trace stats of bench --config CFG
#   pmc:CFG            PMC passes (tools/pmc_pass.sh counter groups) over one bench step of CFG
#   stall:LINE         SQ stall / issue / fetch counters of a bench line (B|C|D|E16k; tools/pmc_stall.sh)
#   prof:CFG           tools/profile_gpu.sh: kernel trace of bench's timed run + PMC passes (traffic) of CFG
#   phase:L,P,N[:KCFG] per-ZMW phase cycle split (tools/phase_prof.py) of N ZMWs of L x P
#   cli:N[:pipe|:fifo] CLI end to end on N config-E ZMWs on stdin, sample vs oracle (tools/cli_stream.py;
#                      pipe: generator piped in, fifo: output through a FIFO)
#   shape:N[:J,J...[:REPS]]  the CLI on N config-E ZMWs at -j J bound to J CPUs (the N = 8 per-rank shape;
#                      SHAPE_TAG names the output directory's suffix)
#   ingest:N           step 0 + prepare alone on N config-E ZMWs (tools/ingest_rate.sh, CPU only)
#   n2:EZMWS           bench.py through torch.distributed.run with two ranks on the box's GPU
#   env:NAME=VALUE     export NAME for the following steps (env:NAME= unsets it)
#   lib:NAME           the following steps load ccsx_amd/NAME (CCSX_LIB); lib: resets
# Environment: CCSX_LIB selects a library variant for the bench steps; CCSX_WG_PER_CU caps the
# resident workgroups per CU (LDS request padding, a measurement hook).
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1

bench_args() {  # CFG [KCFG]
  local a="--config $1 --steps 3 --warmup 1 --no-cpu-baseline --e2e-zmws 0 --e-zmws 0 --roofline-zmws 0"
  [ -n "$2" ] && a="$a --kcfg $2"
  echo "$a"
}

step() {
  local s=$1 name cfg k x
  IFS=: read -r name cfg k x <<< "$s"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1
      local rc=$?; tail -3 "$OUT/gputest.log"; return $rc ;;
    parity)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/parity${CCSX_LIB:+_$CCSX_LIB}.log" 2>&1
      local rc=$?; tail -3 "$OUT/parity${CCSX_LIB:+_$CCSX_LIB}.log"; return $rc ;;
    bench)
      if [ -z "$cfg" ]; then
        timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json"
        return $?
      fi
      local f="$OUT/bench_${cfg}${k:+_k$k}${CCSX_LIB:+_${CCSX_LIB%.so}}${CCSX_WG_PER_CU:+_w$CCSX_WG_PER_CU}.json"
      timeout -k 10 600 python -u bench.py $(bench_args "$cfg" "$k") > "$f" 2> "${f%.json}.err" &&
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], 'ms', d['value'], 'ZMWs/s', d['gcups'], 'GCUPS', 'cfg', d['roofline'].get('kernel_cfg'))" "$f" ;;
    benchn)  # benchn:CFG:N[:KCFG] -- bench.py --config CFG with N ZMWs per GPU
      local f="$OUT/bench_${cfg}_n${k}${x:+_k$x}.json"
      timeout -k 10 600 python -u bench.py $(bench_args "$cfg" "$x") --nzmw "$k" > "$f" 2> "${f%.json}.err" &&
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], 'ms', d['value'], 'ZMWs/s', d['gcups'], 'GCUPS', 'cfg', d['roofline'].get('kernel_cfg'))" "$f" ;;
    ab)  # ab:CFG:KCFG[,KCFG...][:LIB,LIB...] -- 3 interleaved rounds over kernel cfgs x libraries
      local i kk f L libs
      libs=${libs_ab:-libccsx_amd.so}
      [ -n "$x" ] && libs=$x
      for i in 1 2 3; do
        for L in ${libs//,/ }; do
          for kk in ${k//,/ }; do
            f="$OUT/ab_${cfg}_k${kk}_${L%.so}_$i.json"
            CCSX_LIB=$L timeout -k 10 600 python -u bench.py $(bench_args "$cfg" "$kk") > "$f" 2> "${f%.json}.err" || return 1
            python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'k', sys.argv[3], d['ms_per_step'], 'ms', d['gcups'], 'GCUPS')" "$f" "$L" "$kk"
          done
        done
      done ;;
    abx)  # abx:LINE:LIB,LIB... -- 3 interleaved rounds, LINE = B | D | C | E16k (16,384 config-E ZMWs per launch)
      local i f L a
      if [ "$cfg" = E16k ]; then a="--no-kernel-line --roofline-zmws 16384 --steps 3 --warmup 1 --no-cpu-baseline --e2e-zmws 0 --e-zmws 0"
      else a="$(bench_args "$cfg")"; fi
      for i in 1 2 3; do
        for L in ${k//,/ }; do
          f="$OUT/abx_${cfg}_${L%.so}_$i.json"
          CCSX_LIB=$L timeout -k 10 600 python -u bench.py $a > "$f" 2> "${f%.json}.err" || return 1
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], 'ms', d['gcups'], 'GCUPS', d['roofline']['avg_launch_ms'])" "$f" "$L" "$cfg"
        done
      done ;;
    wgcap)  # wgcap:LINE:CAP,CAP... -- the residency curve of a bench line (B|D|E16k) by workgroups per CU
      local i f c a
      if [ "$cfg" = E16k ]; then a="--no-kernel-line --roofline-zmws 16384 --steps 3 --warmup 1 --no-cpu-baseline --e2e-zmws 0 --e-zmws 0"
      else a="$(bench_args "$cfg")"; fi
      for c in ${k//,/ }; do
        f="$OUT/wgcap_${cfg}_w$c.json"
        timeout -k 10 600 python -u bench.py $a --wg-cap "$c" > "$f" 2> "${f%.json}.err" || return 1
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'wg', sys.argv[3], d['ms_per_step'], 'ms', d['gcups'], 'GCUPS')" "$f" "$cfg" "$c"
      done ;;
    e2e)  # e2e:N[:KCFG] -- bench.py's config-E end-to-end line on N ZMWs (CCSX_KCFG forces a kernel cfg)
      local f="$OUT/e2e_${cfg}${k:+_k$k}${CCSX_SHRED_READ_CAP:+_rc$CCSX_SHRED_READ_CAP}.json"
      CCSX_KCFG=${k:--1} CCSX_TIMING=1 timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline \
        --e2e-zmws "$cfg" > "$f" 2> "${f%.json}.err" &&
        python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['e2e']; print(sys.argv[1], d['value'], 'ZMWs/s', d['s'], 's', d['gcups'], 'GCUPS', 'first', d['first_call_s'])" "$f" ;;
    kt)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$cfg" -o kt -- \
        python3 "$R/bench.py" --config "$cfg" --no-cpu-baseline --e2e-zmws 0 --e-zmws 0 --roofline-zmws 0 > "$OUT/kt_$cfg.json" 2> "$OUT/kt_$cfg.err") &&
        echo "kt $cfg done" ;;
    pmc)
      timeout -k 10 900 bash "$R/tools/pmc_pass.sh" "$TAG/pmc_$cfg" --config "$cfg" > "$OUT/pmc_$cfg.log" 2>&1 && echo "pmc $cfg done" ;;
    stall)  # stall:LINE -- SQ stall / issue / fetch counters of a bench line (tools/pmc_stall.sh)
      local d="$OUT/stall_${cfg}${CCSX_LIB:+_${CCSX_LIB%.so}}"
      timeout -k 10 900 bash "$R/tools/pmc_stall.sh" "$d" "$cfg" > "$d.log" 2>&1; local rc=$?
      cat "$d.log"; return $rc ;;
    prof)  # prof:CFG[:N] -- N ZMWs per GPU instead of the config's
      CFG=$cfg NZMW=$k timeout -k 10 1000 bash "$R/tools/profile_gpu.sh" "${TAG}_$cfg${k:+_n$k}" > "$OUT/prof_$cfg.log" 2>&1 && echo "prof $cfg done" ;;
    phase)  # phase:L,PASSES,N:KCFG  (per-ZMW cycle split; CCSX_LIB=libccsx_amd_diag.so for the DP detail)
      local L P N; IFS=, read -r L P N <<< "$cfg"
      timeout -k 10 600 python -u tools/phase_prof.py --L "$L" --passes "$P" --n "$N" --kcfg "${k:--1}" \
        > "$OUT/phase_${L}_${P}_${N}_k${k}${CCSX_LIB:+_$CCSX_LIB}.json" 2> "$OUT/phase.err" &&
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['kernel_ms'],2), 'ms', d['share'], d.get('two_wave'))" "$OUT/phase_${L}_${P}_${N}_k${k}${CCSX_LIB:+_$CCSX_LIB}.json" ;;
    cli)  # cli:N[:pipe] -- tools/cli_stream.py: the CLI on N config-E ZMWs on stdin + oracle sample check
      local tag="cli_$cfg${k:+_$k}${CCSX_SLOTS:+_s$CCSX_SLOTS}${CCSX_CHUNK:+_c$CCSX_CHUNK}${CCSX_CHUNK0:+_f$CCSX_CHUNK0}${CCSX_CTX_BATCHES:+_b$CCSX_CTX_BATCHES}${CCSX_KCFG:+_k$CCSX_KCFG}"
      local flag=""; [ "$k" = pipe ] && flag=--pipe; [ "$k" = fifo ] && flag=--fifo-out
      timeout -k 10 1000 python -u tools/cli_stream.py --n "$cfg" $flag --out "$OUT/$tag" > "$OUT/$tag.log" 2>&1
      local rc=$?; tail -5 "$OUT/$tag.log"; return $rc ;;
    shape)  # shape:N:J,J,... -- the CLI on N config-E ZMWs at -j J bound to J CPUs (tools/rank_shape.py)
      local d="$OUT/shape_$cfg${SHAPE_TAG:+_$SHAPE_TAG}"
      timeout -k 10 900 python -u tools/rank_shape.py --n "$cfg" --jobs "${k:-2,4,8,16}" --repeat "${x:-1}" --out "$d" \
        > "$d.log" 2>&1
      local rc=$?; tail -6 "$d.log"; return $rc ;;
    ingest)  # ingest:N -- step 0 (one reader) + prepare rate on N config-E ZMWs from a file (CPU only)
      timeout -k 10 900 bash tools/ingest_rate.sh "$cfg" 16 "gpurun_out/$TAG" > "$OUT/ingest_$cfg.log" 2>&1
      local rc=$?; tail -2 "$OUT/ingest_$cfg.log"; return $rc ;;
    n2)  # n2:EZMWS -- the driver's two-rank launch on this box (torch.distributed.run, both ranks on its GPU)
      timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --e-zmws "$cfg" --e-sample 100 \
        --nzmw 200 --roofline-zmws 1024 --e2e-zmws 1024 \
        --out-dir "$OUT/n2" > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err"
      local rc=$?; cat "$OUT/bench_n2.json"; return $rc ;;
    env)  # env:NAME=VALUE -- export for the following steps (env:NAME= unsets)
      if [ -n "${cfg#*=}" ]; then export "$cfg"; else unset "${cfg%%=*}"; fi ;;
    lib)  # lib:NAME -- later steps load ccsx_amd/NAME (lib: = the product library)
      if [ -n "$cfg" ]; then export CCSX_LIB=$cfg; else unset CCSX_LIB; fi ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s ($(date +%T))"
  step "$s" || { echo "step $s failed"; exit 1; }
done
echo "session $TAG done"
