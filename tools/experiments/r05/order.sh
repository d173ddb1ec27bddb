cd $GRAFT_REPO_ROOT
O=gpurun_out/order; mkdir -p $O
python3 tools/micro/order_gen.py $O/bin > /dev/null
for r in 1 2; do timeout -k 10 120 tools/micro/loadrun $O/bin/order.hsaco k_scr_rr_d16 k_scr_rr_d48 k_scr_xcd_d16 k_scr_xcd_d48 k_seq_rr_d16 k_seq_rr_d48 k_seq_xcd_d16 k_seq_xcd_d48 k_scr_xcd_d16_p960 k_scr_xcd_d48_p960; done 2>&1 | tee $O/order.txt
