for m in 0x7f 0x77 0x6f 0x5f 0x3f 0x7b 0x7d 0x7e 0x00; do echo "mask $m"; SPWGNN_X6_KERNELS=$m timeout -k 10 100 python3 tools/dbg/step1.py 2>&1 | grep -E "x6: z|x6: logits"; done
