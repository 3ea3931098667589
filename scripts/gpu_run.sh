#!/bin/bash
# One parameterised GPU session (replaces the numbered one-off scripts of round 3).
# usage: bash scripts/gpu_run.sh TAG STEP [STEP ...]
#   pmc        PMC HBM passes of the C3 headline and the weak8 share -> profiles/TAG_traffic*.json
#   tests=EXPR pytest -m gpu -k EXPR (EXPR "all": every gpu test)
#   prof[m]    rocprofv3 --kernel-trace --stats of the headline -> gpurun_out/prof[m]_TAG (m: mirror)
#   bench      the default bench line (CPU baseline, weak8, strong C4, proxies fast)
#   benchall   the default bench line with --proxy all (adds C5 on 8 ranks and C5 on one GPU)
#   hl, hl2    headline only, no CPU baseline (--streams 1 / 2), mirror mode forced off: quick A/B lines
#   hlm        the same with the mirror mode forced on (the float32 default)
#   configs    bench.py --config C2 C3 C4 C5s
#   smoke      __graft_entry__.smoke()
# Every step has its own time limit; the first failing step ends the session.
set -u
mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  return $rc
}
for step in "$@"; do
  case $step in
    pmc)
      run pmc_c3 400 bash scripts/pmc.sh ${TAG} > gpurun_out/pmc_${TAG}.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}.log; exit 1; }
      cp gpurun_out/${TAG}_traffic.json profiles/${TAG}_traffic.json
      WORKLOAD=weak8 run pmc_weak8 400 bash scripts/pmc.sh ${TAG}w8 > gpurun_out/pmc_${TAG}w8.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}w8.log; exit 1; }
      cp gpurun_out/${TAG}w8_traffic.json profiles/${TAG}_traffic_weak8.json
      tail -12 gpurun_out/pmc_${TAG}.log ;;
    sq|sqm)  # FETCH_SIZE + SQ counters of the headline (scripts/passes_fwd_sq.txt); m: mirror mode
      mm=0; [ $step = sqm ] && mm=1
      ADMM_FWD_MIRROR=$mm PASSFILE=scripts/passes_fwd_sq.txt run $step 600 bash scripts/pmc.sh ${step}_${TAG} > gpurun_out/${step}_${TAG}.log 2>&1 || { tail -5 gpurun_out/${step}_${TAG}.log; exit 1; }
      python scripts/pmc_summary.py ${step}_${TAG} "k_fwdg<" "k_back" ;;
    sq5)  # SQ counters (scripts/passes_sq_r5.txt: issue, LDS, wait, f64 / cvt counts) of the C3 headline, default modes
      PASSFILE=scripts/passes_sq_r5.txt run sq5 600 bash scripts/pmc.sh sq5_${TAG} > gpurun_out/sq5_${TAG}.log 2>&1 || { tail -5 gpurun_out/sq5_${TAG}.log; exit 1; }
      python scripts/pmc_summary.py sq5_${TAG} "k_fwdg<" "k_back_mirror_2<float, 8, 4>" "k_back_mirror<float, 8, 4, 3>" "k_tv_update<float, 4, false, true, true, true>" "k_cg_update<float, 4, true, false>" | tee gpurun_out/sq5_${TAG}_summary.txt ;;
    tvc)  # round 6: TA / TCP / TCC / TD / SQ counters of the TV and CG updates (scripts/passes_tv_r6.txt)
      PASS_TIMEOUT=150 PASSFILE=scripts/passes_tv_r6.txt run tvc 700 bash scripts/pmc.sh tvc_${TAG} > gpurun_out/tvc_${TAG}.log 2>&1 || { tail -5 gpurun_out/tvc_${TAG}.log; exit 1; }
      python scripts/pmc_summary.py tvc_${TAG} "k_tv_update<float, 4, false, true, true, true>" "k_cg_update<float, 4, true, false>" "k_back_mirror_2<float, 8, 4>" | tee gpurun_out/tvc_${TAG}_summary.txt ;;
    tests=*)
      expr=${step#tests=}
      if [ "$expr" = all ]; then k=(); else k=(-k "$expr"); fi
      # -s: tests that run minutes (the 20-iteration C3 oracle) print progress lines to the log
      run pytest 700 python -u -m pytest tests -m gpu "${k[@]}" -v -s -rf --timeout 600 --timeout-method thread --durations=15 > gpurun_out/pytest_${TAG}.log 2>&1
      rc=$?; tail -25 gpurun_out/pytest_${TAG}.log; [ $rc -ne 0 ] && exit $rc ;;
    etests=*)  # etests=VAR=VAL:EXPR -- pytest -m gpu -k EXPR with VAR=VAL in the environment (A/B of a kernel switch)
      v=${step#etests=}; kv=${v%%:*}; expr=${v#*:}
      env "$kv" timeout -k 10 1100 python -u -m pytest tests -m gpu -k "$expr" -v -s -rf --timeout 900 --timeout-method thread > gpurun_out/etests_${TAG}.log 2>&1
      rc=$?; tail -15 gpurun_out/etests_${TAG}.log; [ $rc -ne 0 ] && exit $rc ;;
    envhl=*)  # envhl=VAR=VAL[@WORKLOAD]: headline only (no CPU baseline) with VAR=VAL in the environment
      v=${step#envhl=}; wl=C3; case $v in *@*) wl=${v#*@}; v=${v%@*} ;; esac
      nm=$(echo "$v" | tr '=' '_')
      env "$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only --workload $wl > gpurun_out/envhl_${nm}_${wl}_${TAG}.json 2> gpurun_out/envhl_${nm}_${wl}_${TAG}.err || { tail -5 gpurun_out/envhl_${nm}_${wl}_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/envhl_${nm}_${wl}_${TAG}.json ;;
    prof|profm|profd)  # prof: default modes; profm / profd: mirror-mode forward forced on / off
      mm=; [ $step = profm ] && mm=1; [ $step = profd ] && mm=0
      ADMM_FWD_MIRROR=$mm run $step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${step}_${TAG} -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --headline-only > gpurun_out/${step}_${TAG}.log 2>&1 || exit 1
      python scripts/top_kernels.py gpurun_out/${step}_${TAG} ;;
    profvar=*)  # profvar=NAME: rocprofv3 kernel stats of the headline with variants/lib_NAME.so ("base": in-tree)
      v=${step#profvar=}; lib=variants/lib_$v.so; [ $v = base ] && lib=
      ADMM_TOMO_LIB=$lib run $step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profvar_${v}_${TAG} -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --headline-only > gpurun_out/profvar_${v}_${TAG}.log 2>&1 || exit 1
      python scripts/top_kernels.py gpurun_out/profvar_${v}_${TAG} > gpurun_out/profvar_${v}_${TAG}.txt; head -8 gpurun_out/profvar_${v}_${TAG}.txt ;;
    bench)
      run bench 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -5 gpurun_out/bench_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/bench_${TAG}.json ;;
    benchall)
      run benchall 900 python bench.py --steps 20 --warmup 5 --proxy all > gpurun_out/benchall_${TAG}.json 2> gpurun_out/benchall_${TAG}.err || { tail -5 gpurun_out/benchall_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/benchall_${TAG}.json ;;
    hl|hl2|hl4|hlm|hlm2)  # quick headline A/B (no CPU baseline): --streams 1/2/4; m = ADMM_FWD_MIRROR=1
      st=1; case $step in *2) st=2 ;; *4) st=4 ;; esac
      mm=0; case $step in hlm*) mm=1 ;; esac
      ADMM_FWD_MIRROR=$mm run $step 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only --streams $st > gpurun_out/${step}_${TAG}.json 2> gpurun_out/${step}_${TAG}.err || { tail -5 gpurun_out/${step}_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/${step}_${TAG}.json ;;
    var=*)  # var=NAME[@WORKLOAD]: headline (C3 or weak8) with the tuning build variants/lib_NAME.so
            # (scripts/sweep_build.py; NAME "base": the in-tree library), default modes
      v=${step#var=}; wl=C3; case $v in *@*) wl=${v#*@}; v=${v%@*} ;; esac
      lib=variants/lib_$v.so; [ $v = base ] && lib=
      ADMM_TOMO_LIB=$lib run $step 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only --workload $wl > gpurun_out/var_${v}_${wl}_${TAG}.json 2> gpurun_out/var_${v}_${wl}_${TAG}.err || { tail -5 gpurun_out/var_${v}_${wl}_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/var_${v}_${wl}_${TAG}.json ;;
    plan=*)  # plan=K[:m]: headline with the forward plan forced to K (ADMM_FWD_PLAN; m: mirror mode)
      v=${step#plan=}; mm=0; case $v in *:m) mm=1; v=${v%:m} ;; esac
      ADMM_FWD_PLAN=$v ADMM_FWD_MIRROR=$mm run $step 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only > gpurun_out/plan_${v}_${mm}_${TAG}.json 2> gpurun_out/plan_${v}_${mm}_${TAG}.err || { tail -5 gpurun_out/plan_${v}_${mm}_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/plan_${v}_${mm}_${TAG}.json ;;
    benchallm)  # benchall with the mirror-mode forward
      ADMM_FWD_MIRROR=1 run benchallm 900 python bench.py --steps 20 --warmup 5 --proxy all --no-cpu-baseline > gpurun_out/benchallm_${TAG}.json 2> gpurun_out/benchallm_${TAG}.err || { tail -5 gpurun_out/benchallm_${TAG}.err; exit 1; }
      python scripts/summarize_bench.py gpurun_out/benchallm_${TAG}.json ;;
    share=*)  # share=CONFIG:R/W[:d]: one rank's share on this GPU (bench --as-rank; d: --edge-state derived A/B)
      v=${step#share=}; cfg=${v%%:*}; rest=${v#*:}; rw=${rest%%:*}; sz=()
      case $rest in *:d) sz=(--edge-state derived) ;; esac
      out=gpurun_out/share_${cfg}_${rw/\//of}${sz:+_z}_${TAG}.json
      run $step 600 python bench.py --config $cfg --as-rank $rw --steps 4 --warmup 2 "${sz[@]}" > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
      tail -c 600 $out ;;
    bitwise=*)  # bitwise=NAME[:N]: scripts/check_bitwise.py with the in-tree library and variants/lib_NAME.so
      v=${step#bitwise=}; n=64; case $v in *:*) n=${v#*:}; v=${v%%:*} ;; esac
      CHECK_N=$n run bw_base 300 python scripts/check_bitwise.py gpurun_out/bw_base_${n}_${TAG}.npz > gpurun_out/bw_${v}_${n}_${TAG}.log 2>&1 &&
      CHECK_N=$n ADMM_TOMO_LIB=variants/lib_$v.so run bw_$v 300 python scripts/check_bitwise.py gpurun_out/bw_${v}_${n}_${TAG}.npz >> gpurun_out/bw_${v}_${n}_${TAG}.log 2>&1 ||
        { tail -5 gpurun_out/bw_${v}_${n}_${TAG}.log; exit 1; }
      python scripts/check_bitwise.py --compare gpurun_out/bw_base_${n}_${TAG}.npz gpurun_out/bw_${v}_${n}_${TAG}.npz ;;
    configs)
      run configs 1000 bash scripts/run_configs.sh C2 C3 C4 C5s || exit 1 ;;
    smoke)
      run smoke 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_${TAG}.log 2>&1
      rc=$?; tail -2 gpurun_out/smoke_${TAG}.log; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
