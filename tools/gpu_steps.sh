# GPU steps on one MI355X, chosen by RUNS (space-separated): sgemv sgprobe sgprobe0 mfma0b8 b4m3 b16 b4 b8 arr3 sg0b8 proffp8b64 selflaunch
# tests ktests recov mg smoke bench fp8 fp8loop ab n256 n256w4 gmm prio tp2 tp8 pf8 loopprobe prof proffp8 fp8head loopbf wide merge swl b8b b64 tp8b64 tp8plain ab8b tune8b proftp8 fp8tp4 tunefp8 minmi
# attn kbattn attntr chain.
# Each GPU step has its own time limit; test failures (rc 1) do not stop later steps, a timeout / abort / fault
# (any other rc) ends the script.  Logs land in gpurun_out/$OUT (default r4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-r4}; mkdir -p $O
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$O/$log"; exit $rc; fi
  return 0
}
for spec in ${RUNS:-tests smoke bench}; do
  case $spec in
    attn) step 300 attn_tests.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode_attention" --timeout 120 --timeout-method thread
          tail -3 $O/attn_tests.log ;;
    kbattn) for m in 4 8 16 64; do step 200 kb_attn_m$m.txt python -u tools/kbench.py --tp 1 --M $m
              grep -h "decode_attn" $O/kb_attn_m$m.txt | sed "s/^/M=$m /"; done
            step 200 kb_attn_tp8_m64.txt python -u tools/kbench.py --tp 8 --M 64
            grep -h "decode_attn" $O/kb_attn_tp8_m64.txt | sed "s/^/tp8 M=64 /" ;;
    kbattn512) for m in 8 16 64; do K8S_ATTN_FUSED_PART=512 step 200 kb_attn512_m$m.txt python -u tools/kbench.py --tp 1 --M $m
                 grep -h "decode_attn\[one-wg\]" $O/kb_attn512_m$m.txt | sed "s/^/part512 M=$m /"; done
               K8S_ATTN_FUSED_PART=512 step 200 kb_attn512_tp8_m64.txt python -u tools/kbench.py --tp 8 --M 64
               grep -h "decode_attn\[one-wg\]" $O/kb_attn512_tp8_m64.txt | sed "s/^/part512 tp8 M=64 /" ;;
    mgab) i=0; for ov in "" ${MGOV:-}; do i=$((i+1)); K8S_MGEMM_OVERRIDE="$ov" step 400 bench_b64_ov$i.json python -u bench.py --batch 64 --steps 2 --warmup 1
            echo "override [$ov]: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_b64_ov$i.json | tr '\n' ' ')"; done ;;
    rmsab) for i in 1 2; do for um in 0 64; do K8S_RMS_UNFUSED_MAX_M=$um step 400 bench_b64_rms$um.json python -u bench.py --batch 64 --steps 2 --warmup 1
             echo "unfused<=$um: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*' $O/bench_b64_rms$um.json | tr '\n' ' ')"; done; done ;;
    rmsab2) for um in 0 64; do K8S_RMS_UNFUSED_MAX_M=$um step 400 bench_b32_rms$um.json python -u bench.py --batch 32 --steps 2 --warmup 1
             echo "b32 unfused<=$um: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*' $O/bench_b32_rms$um.json | tr '\n' ' ')"; done
            for um in 0 256; do K8S_RMS_UNFUSED_MAX_M=$um step 400 bench_def_rms$um.json python -u bench.py --steps 6 --warmup 2
             echo "default unfused<=$um: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_def_rms$um.json | tr '\n' ' ')"; done ;;
    wgab) for i in 1 2; do for wg in 1 2; do K8S_SGEMV_WG_PER_CU=$wg step 400 bench_b8_wg$wg.json python -u bench.py --batch 8 --steps 4 --warmup 1
             echo "b8 wg/cu=$wg: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*' $O/bench_b8_wg$wg.json | tr '\n' ' ')"; done; done ;;
    chain) step 120 chain_probe.txt python -u tools/probes/chain_probe.py
           cat $O/chain_probe.txt
           step 120 chain_probe_pre2.txt python -u tools/probes/chain_probe.py chain_pre2.so
           cat $O/chain_probe_pre2.txt ;;
    rowslab) step 300 pgemm_tests.log python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 200 --timeout-method thread
             tail -3 $O/pgemm_tests.log
             for i in 1 2; do for rs in 0 1; do K8S_PGEMM_ROWSLAB=$rs step 400 bench_def_rs$rs.json python -u bench.py --steps 6 --warmup 2
               echo "default rowslab=$rs: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_def_rs$rs.json | tr '\n' ' ')"; done; done ;;
    gemmtests) step 400 gemm_tests.log python -u -m pytest tests/test_pgemm_gpu.py tests/test_mgemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread
               tail -3 $O/gemm_tests.log ;;
    mgemm_ab) for i in 1 2; do step 400 bench_b64_$i.json python -u bench.py --batch 64 --steps 2 --warmup 1
                echo "b64 run $i: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_b64_$i.json | tr '\n' ' ')"
                step 400 bench_tp8b64_$i.json python -u bench.py --simulate-tp 8 --batch 64 --steps 3 --warmup 1
                echo "tp8sim b64 run $i: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_tp8b64_$i.json | tr '\n' ' ')"; done ;;
    rsab2) for rs in 1 0 1 0; do K8S_PGEMM_ROWSLAB=$rs step 400 bench_tp8b64_rs$rs.json python -u bench.py --simulate-tp 8 --batch 64 --steps 3 --warmup 1
             echo "tp8sim b64 rowslab=$rs: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_tp8b64_rs$rs.json | tr '\n' ' ')"
             K8S_PGEMM_ROWSLAB=$rs step 400 bench_b64_rs$rs.json python -u bench.py --batch 64 --steps 2 --warmup 1
             echo "b64 rowslab=$rs: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_b64_rs$rs.json | tr '\n' ' ')"
             K8S_PGEMM_ROWSLAB=$rs step 400 bench_tp8_rs$rs.json python -u bench.py --simulate-tp 8 --steps 6 --warmup 2
             echo "tp8sim rowslab=$rs: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_tp8_rs$rs.json | tr '\n' ' ')"; done ;;
    rmsab3) for um in 0 64 0 64; do K8S_RMS_UNFUSED_MAX_M=$um step 400 bench_tp8b64_um$um.json python -u bench.py --simulate-tp 8 --batch 64 --steps 3 --warmup 1
             echo "tp8sim b64 unfused<=$um: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_tp8b64_um$um.json | tr '\n' ' ')"
             K8S_RMS_UNFUSED_MAX_M=$um step 400 bench_b64_um$um.json python -u bench.py --batch 64 --steps 2 --warmup 1
             echo "b64 unfused<=$um: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*' $O/bench_b64_um$um.json | tr '\n' ' ')"; done ;;
    ptune256) step 900 ptune256.txt python -u tools/pgemm_tune.py --tp 1 --m 256 --write --json-out $O/ptune256.json
              cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json $O/pgemm_gfx950_tuned.json
              tail -12 $O/ptune256.txt
              step 400 bench_default_tuned.json python -u bench.py --steps 6 --warmup 2
              echo "default with the re-tuned 256-row plans: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_default_tuned.json | tr '\n' ' ')" ;;
    ptunewide) step 1100 ptunewide.txt python -u tools/pgemm_tune.py --tp 1 8 4 --m 192 256 320 384 512 768 1024 2048 8192 --write --json-out $O/ptunewide.json
               cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json $O/pgemm_gfx950_wide.json
               grep "pgemm >= library" $O/ptunewide.txt ;;
    ptunefp8) step 1100 ptunefp8.txt python -u tools/pgemm_tune.py --fp8 --tp 1 4 --m 192 256 320 384 512 --write --json-out $O/ptunefp8.json
              cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json $O/pgemm_gfx950_fp8.json
              grep "pgemm >= library" $O/ptunefp8.txt
              step 400 bench_fp8_tuned.json python -u bench.py --dtype fp8 --steps 6 --warmup 2
              echo "fp8 with the re-tuned plans: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_fp8_tuned.json | tr '\n' ' ')" ;;
    n256ab) # prev: a table file placed at tmp_ab/pgemm_prev.json before the call (e.g. git show <rev>:<table>)
            for v in cur rs0 prev cur; do
              [ $v = prev ] && [ ! -f tmp_ab/pgemm_prev.json ] && continue
              case $v in cur) E="";; rs0) E="K8S_PGEMM_ROWSLAB=0";; prev) E="K8S_PGEMM_TABLE_PATH=$GRAFT_REPO_ROOT/tmp_ab/pgemm_prev.json";; esac
              env $E timeout -k 10 400 python -u bench.py --nodes 256 --max-model-len 32768 --steps 3 --warmup 1 > $O/n256_$v.json 2>&1 || { tail -5 $O/n256_$v.json; exit 1; }
              echo "n256 $v: $(grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/n256_$v.json | tr '\n' ' ')"; done ;;
    pfattn) step 300 pfattn_tests.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k "prefill" --timeout 120 --timeout-method thread
            tail -2 $O/pfattn_tests.log
            bash tools/gpu_prof.sh tp1_default_pf "" > $O/prof_pf.log 2>&1 || { tail -20 $O/prof_pf.log; exit 1; }
            grep -A12 "last prefill" gpurun_out/lastfwd_tp1_default_pf.txt ;;
    redab) step 300 pgemm_tests.log python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 200 --timeout-method thread
           tail -2 $O/pgemm_tests.log
           bash tools/gpu_prof.sh tp1_default_red "" > $O/prof_red.log 2>&1 || { tail -20 $O/prof_red.log; exit 1; }
           grep -A12 "last prefill" gpurun_out/lastfwd_tp1_default_red.txt ;;
    awab) for aw in 0 8 0 8; do K8S_PREFILL_ATTN_WAVES=$aw step 400 bench_def_aw$aw.json python -u bench.py --steps 6 --warmup 2
            echo "default attn waves=$aw: $(grep -ho '"value": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_def_aw$aw.json | tr '\n' ' ')"; done
          for aw in 0 4; do K8S_PREFILL_ATTN_WAVES=$aw step 400 bench_n256_aw$aw.json python -u bench.py --nodes 256 --max-model-len 32768 --steps 3 --warmup 1
            echo "n256 attn waves=$aw: $(grep -ho '"value": [0-9.]*\|"prefill_ms_per_decision": [0-9.]*' $O/bench_n256_aw$aw.json | tr '\n' ' ')"; done ;;
    mgtune64) step 300 mgtune64.txt python -u tools/mgemm_tune.py --tp 1 --m 64 --only ${MGONLY:-qkv o_proj} --verbose
              tail -40 $O/mgtune64.txt ;;
    attntr) step 200 attn_trace.txt python -u tools/attn_trace.py ;;
    attnqb) for v in 32 "" 32 ""; do step 200 attn_trace_qb$v.txt python -u tools/attn_trace.py attn_trace$v.so
              echo "== merge batch ${v:-36} lanes"; grep -A1 "TP=8 ctx=  564\|TP=1 ctx=  564 pmax= 9" $O/attn_trace_qb$v.txt | grep -v "^--"; done ;;
    sgemv) step 300 sgemv_tests.log python -u -m pytest tests/test_sgemv_gpu.py -x -q --timeout 200 --timeout-method thread
           tail -3 $O/sgemv_tests.log ;;
    sgprobe) step 300 sgemv_probe.txt python -u tools/sgemv_probe.py 5
           grep -v amdgpu.ids $O/sgemv_probe.txt ;;
    sgprobe0) K8S_SGEMV_MFMA_MIN_M=17 step 300 sgemv_probe_nomfma.txt python -u tools/sgemv_probe.py 5
           grep -v amdgpu.ids $O/sgemv_probe_nomfma.txt | grep M=8 ;;
    mfma0b8) K8S_SGEMV_MFMA_MIN_M=17 step 400 bench_b8_nomfma.json python -u bench.py --batch 8 --steps 4 --warmup 1
           grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*' $O/bench_b8_nomfma.json | tr '\n' ' '; echo " (batch 8, sgemv v_dot2 form)" ;;
    b4m3) K8S_SGEMV_MFMA_MIN_M=3 step 400 bench_b4_mfma.json python -u bench.py --batch 4 --steps 4 --warmup 1
           grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*' $O/bench_b4_mfma.json | tr '\n' ' '; echo " (batch 4, sgemv MFMA form)" ;;
    b16) step 400 bench_b16.json python -u bench.py --batch 16 --steps 4 --warmup 1
           grep -h '"metric"' $O/bench_b16.json | cut -c1-300; grep -ho '"decode_ms_per_step": [0-9.]*' $O/bench_b16.json ;;
    b4) step 400 bench_b4.json python -u bench.py --batch 4 --steps 4 --warmup 1
           grep -h '"metric"' $O/bench_b4.json | cut -c1-300; grep -ho '"decode_ms_per_step": [0-9.]*' $O/bench_b4.json ;;
    b8) step 400 bench_b8.json python -u bench.py --batch 8 --steps 4 --warmup 1
           grep -h '"metric"' $O/bench_b8.json | cut -c1-300; grep -ho '"decode_ms_per_step": [0-9.]*' $O/bench_b8.json ;;
    sg0b8) for b in 4 8; do K8S_SGEMV=0 step 400 bench_b${b}_nosgemv.json python -u bench.py --batch $b --steps 4 --warmup 1
           grep -ho '"value": [0-9.]*\|"decode_ms_per_step": [0-9.]*' $O/bench_b${b}_nosgemv.json | tr '\n' ' '; echo " (batch $b, mgemm)"; done ;;
    arr3) step 600 bench_arrivals3.json python -u bench.py --arrival-rate 3 --batch 16 --steps 40 --warmup 4
           grep -h '"metric"' $O/bench_arrivals3.json | cut -c1-900 ;;
    proffp8b64) bash tools/gpu_prof.sh tp1_fp8_b64 "--dtype fp8 --batch 64" > $O/proffp8b64.log 2>&1 || { tail -20 $O/proffp8b64.log; exit 1; }
          head -24 gpurun_out/rocprof_70b_tp1_fp8_b64_kernels.txt ;;
    selflaunch) step 600 selflaunch.log python -u -m pytest tests/test_multigpu.py -x -q -k "self_launch or share_one_gpu" --timeout 500 --timeout-method thread
           tail -3 $O/selflaunch.log ;;
    tests) step 600 gputests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
           tail -3 $O/gputests.log ;;
    ktests) step 300 ktests.log python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
           tail -3 $O/ktests.log ;;
    smoke) step 180 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
           tail -1 $O/smoke.log | cut -c1-300 ;;
    bench) step 400 bench_default.json python -u bench.py --steps 8 --warmup 2
           grep -h '"metric"' $O/bench_default.json | cut -c1-600 ;;
    fp8) step 400 bench_fp8.json python -u bench.py --dtype fp8 --steps 6 --warmup 2
           grep -h '"metric"' $O/bench_fp8.json | cut -c1-600 ;;
    fp8loop) K8S_GEMV_LOOP=${LOOPWG:-4} step 400 bench_fp8_loop.json python -u bench.py --dtype fp8 --steps 6 --warmup 2
           grep -h '"metric"' $O/bench_fp8_loop.json | cut -c1-600 ;;
    recov) step 200 recovery.log python -u -m pytest tests/test_recovery_gpu.py -x -q -s --timeout 180 --timeout-method thread
           grep -E "recovery trace|passed|failed" $O/recovery.log | cut -c1-3000 ;;
    ab) for i in 1 2; do for lw in 0 ${LOOPWG:-2}; do
          K8S_GEMV_LOOP=$lw step 400 ab_${AB_TAG:-fp8}_loop${lw}_$i.json python -u bench.py ${AB_ARGS:---dtype fp8} --steps 6 --warmup 2
          grep -h '"metric"' $O/ab_${AB_TAG:-fp8}_loop${lw}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('loop=$lw', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'), d.get('init_s'))"
        done; done ;;
    mg) step 500 multigpu.log python -u -m pytest tests/test_multigpu.py -x -q -s --timeout 480 --timeout-method thread
           grep -E "rehearsal|passed|failed" $O/multigpu.log | cut -c1-600 ;;
    n256) step 400 bench_nodes256.json python -u bench.py --nodes 256 --max-model-len 32768 --steps 3 --warmup 1
           grep -h '"metric"' $O/bench_nodes256.json | cut -c1-200; grep -ho '"decode_ms_per_step[^}]*prefill_tokens_per_decision": [0-9.]*' $O/bench_nodes256.json ;;
    n256w4) K8S_PREFILL_ATTN_WAVES=${AW:-4} step 400 bench_nodes256_w4.json python -u bench.py --nodes 256 --max-model-len 32768 --steps 3 --warmup 1
           grep -h '"metric"' $O/bench_nodes256_w4.json | cut -c1-200; grep -ho '"decode_ms_per_step[^}]*prefill_tokens_per_decision": [0-9.]*' $O/bench_nodes256_w4.json ;;
    tp2) STEPS=3 step 900 tp2_rehearsal.log bash tools/gpu_tp2_rehearsal.sh
           tail -3 $O/tp2_rehearsal.log | cut -c1-700 ;;
    gmm) for b in ${GMM_B:-4 8}; do for mm in 2 8; do
          K8S_GEMV_MAX_M=$mm step 400 gmm_b${b}_m${mm}.json python -u bench.py --batch $b --steps 3 --warmup 1
          grep -h '"metric"' $O/gmm_b${b}_m${mm}.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch $b gemv_max_m=$mm', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    prio) step 500 pgemm_prio_probe.txt python -u tools/pgemm_prio_probe.py --m 256 2048 8192
           grep -v amdgpu.ids $O/pgemm_prio_probe.txt ;;
    fp8head) for i in 1 2; do for h in 0 1; do
          K8S_FP8_LM_HEAD=$h step 400 fp8head${h}_$i.json python -u bench.py --dtype fp8 --steps 6 --warmup 2
          grep -h '"metric"' $O/fp8head${h}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fp8 lm_head=$h', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    loopbf) for i in 1 2; do for lw in 0 2 4; do
          K8S_GEMV_LOOP_BF16=$lw step 400 loopbf${lw}_$i.json python -u bench.py --steps 6 --warmup 2
          grep -h '"metric"' $O/loopbf${lw}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16 plain-epilogue loop=$lw', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    wide) for i in 1 2; do for wd in 0 1; do
          K8S_GEMV_WIDE=$wd step 400 wide${wd}_$i.json python -u bench.py --steps 6 --warmup 2
          grep -h '"metric"' $O/wide${wd}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16 gemv wide=$wd', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    merge) for i in 1 2; do for mw in 0 1; do
          K8S_ATTN_MERGE_WIDE=$mw step 300 merge${mw}_$i.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2
          grep -h '"metric"' $O/merge${mw}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tp8sim merge_wide=$mw', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    swl) for i in 1 2; do for sm in 0 2048; do
          K8S_GEMV_LOOP_SWIGLU_MAX=$sm step 300 swl${sm}_$i.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2
          grep -h '"metric"' $O/swl${sm}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tp8sim swiglu_loop_max=$sm', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    b8b) step 300 bench_8b.json python -u bench.py --preset llama-3-8b --steps 10 --warmup 2
           grep -h '"metric"' $O/bench_8b.json | cut -c1-300 ;;
    b64) step 400 bench_b64.json python -u bench.py --batch 64 --steps 2 --warmup 1
           grep -h '"metric"' $O/bench_b64.json | cut -c1-300 ;;
    tp8b64) step 400 bench_tp8sim_b64.json python -u bench.py --simulate-tp 8 --batch 64 --steps 3 --warmup 1
           grep -h '"metric"' $O/bench_tp8sim_b64.json | cut -c1-300 ;;
    tp8plain) K8S_GEMV_LOOP_BF16=0 step 300 bench_tp8sim_noplainloop.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2
           grep -h '"metric"' $O/bench_tp8sim_noplainloop.json | cut -c1-200; grep -ho '"decode_ms_per_step": [0-9.]*' $O/bench_tp8sim_noplainloop.json ;;
    ab8b) for i in 1 2; do for lw in 0 2; do
          K8S_GEMV_LOOP_BF16=$lw step 300 ab8b_loop${lw}_$i.json python -u bench.py --preset llama-3-8b --steps 10 --warmup 2
          grep -h '"metric"' $O/ab8b_loop${lw}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('8b plain loop=$lw', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    tune8b) step 900 tune8b.txt python -u tools/pgemm_tune.py --model 8b --tp 1 --m 256 512 2048 8192 --only qkv o_proj gate_up down --write --json-out $O/tune8b.json
           grep -v amdgpu.ids $O/tune8b.txt | tail -20; cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json $O/pgemm_gfx950.json ;;
    proftp8) bash tools/gpu_prof.sh tp8sim "--simulate-tp 8" > $O/proftp8.log 2>&1 || { tail -20 $O/proftp8.log; exit 1; }
          grep -A12 "last decode" gpurun_out/lastfwd_tp8sim.txt ;;
    fp8tp4) step 300 bench_fp8_tp4sim.json python -u bench.py --dtype fp8 --simulate-tp 4 --steps 10 --warmup 2
           grep -h '"metric"' $O/bench_fp8_tp4sim.json | cut -c1-200; grep -ho '"decode_ms_per_step": [0-9.]*, "prefill_ms_per_step": [0-9.]*' $O/bench_fp8_tp4sim.json ;;
    tunefp8) step 1100 tunefp8.txt python -u tools/pgemm_tune.py --fp8 --tp 1 4 --m 192 256 384 512 768 1024 2048 4096 8192 --only qkv o_proj gate_up down --write --json-out $O/tunefp8.json
           grep -v amdgpu.ids $O/tunefp8.txt | tail -8; cp k8s_llm_scheduler_amd/engine/assets/pgemm_gfx950.json $O/pgemm_gfx950.json ;;
    minmi) for i in 1 2; do for mm in ${MINMI:-64 65}; do
          K8S_GEMV_LOOP_MIN_MI=$mm step 400 minmi${mm}_$i.json python -u bench.py --steps 8 --warmup 2 ${MINMI_ARGS:-}
          grep -h '"metric"' $O/minmi${mm}_$i.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16 loop_min_mi=$mm', d['value'], d.get('decode_ms_per_step'), d.get('prefill_ms_per_decision'))"
        done; done ;;
    tp8) step 300 bench_tp8sim.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2
           grep -h '"metric"' $O/bench_tp8sim.json | cut -c1-600 ;;
    pf8) K8S_DECODE_PREFETCH_MB=${PFMB:-24} step 300 bench_tp8sim_pf.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2
           grep -h '"metric"' $O/bench_tp8sim_pf.json | cut -c1-600 ;;
    loopprobe) step 400 gemv_loop_probe.txt python -u tools/gemv_loop_probe.py --tp 1 4 8
           cat $O/gemv_loop_probe.txt | grep -v amdgpu.ids ;;
    proffp8) bash tools/gpu_prof.sh tp1_fp8 "--dtype fp8" > $O/proffp8.log 2>&1 || { tail -20 $O/proffp8.log; exit 1; }
          head -20 gpurun_out/rocprof_70b_tp1_fp8_kernels.txt; cat gpurun_out/lastfwd_tp1_fp8.txt ;;
    prof) bash tools/gpu_prof.sh tp1_default "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
          head -24 gpurun_out/rocprof_70b_tp1_default_kernels.txt ;;
  esac
done
