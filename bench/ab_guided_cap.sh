# config 5: steps that decode guided (tool-call) rows carry at most CAP prefill tokens (B)
# vs the normal 512-row soft budget (A).  Summary: bench/bsum.py over the four logs.
S5="python bench.py --agent-tools 0.2 --steps 20 --warmup 5"
bash gpurun_step.sh "gcA1:400:ENGINE_GUIDED_PREFILL_CAP=0 $S5" "gcB1:400:ENGINE_GUIDED_PREFILL_CAP=${CAP:-96} $S5" \
  "gcA2:400:ENGINE_GUIDED_PREFILL_CAP=0 $S5" "gcB2:400:ENGINE_GUIDED_PREFILL_CAP=${CAP:-96} $S5"
