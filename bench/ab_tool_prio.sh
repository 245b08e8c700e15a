# config 5: tool-round follow-up prefilled at arrival order (A) vs ahead of waiting prompts (B)
S5="python bench.py --agent-tools 0.2 --steps 20 --warmup 5"
bash gpurun_step.sh "tpA1:400:AGENT_TOOL_ROUND_PRIORITY=0 $S5" "tpB1:400:$S5" "tpA2:400:AGENT_TOOL_ROUND_PRIORITY=0 $S5" "tpB2:400:$S5"
