for d in 0 1 2 3 7; do YH_CK_DBG=$d timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 2>&1 | grep " c3k " | head -1 | sed "s/^/dbg$d /"; done
