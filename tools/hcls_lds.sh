# fused head cls: phase trace under several tile LDS budgets (YH_HCLS_LDS)
for b in "$@"; do echo "budget $b"; YH_HCLS_LDS=$b timeout -k 10 200 python tools/hcls_trace.py 2>&1 | grep head_cls | tail -1; done
