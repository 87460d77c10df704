for k in 0 512 1024 1536 776 1032; do echo "knob $k"; QTX_ATTN_KNOB=$k timeout -k 10 100 python tools/attn_bench.py 2>&1 | grep quant || exit 1; done
