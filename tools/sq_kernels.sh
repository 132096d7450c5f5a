#!/bin/bash
# SALU / VALU issue balance of the bootstrap and step kernels other than k_lk_w (one --pmc pass
# of the headline bench): sq_kernels.sh <tag> [kernel regex]
export TMPDIR=/tmp
O=gpurun_out; tag=$1; KR=${2:-"k_sift_desc_w|k_sift_ori|k_eig3|k_pnp_tri|k_essential|k_blur_tile_n|k_extrema_t|k_gsel_walk|k_add_finish_lean|k_pyr_rows"}
HL="--no-cpu --no-single --no-match --no-sequence"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --kernel-include-regex "$KR" --output-format csv -d $O/sqk_$tag -o run -- python bench.py $HL --steps 5 --warmup 2 > $O/sqk_$tag.json 2>&1 || exit $?
python3 - "$O/sqk_$tag" <<'PY'
import csv, glob, re, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(lambda: defaultdict(int))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:30]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CU_CYCLES", 0)):
    busy = c.get("SQ_BUSY_CU_CYCLES", 0)
    if not busy: continue
    salu = c.get("SQ_INST_CYCLES_SALU", 0) / busy
    valu = c.get("SQ_INSTS_VALU", 0) * 2 / 4 / busy
    print(f"{k:24s} launches {n[k]['SQ_BUSY_CU_CYCLES']:4d} busy {busy/256/2.4e3/max(1,n[k]['SQ_BUSY_CU_CYCLES']):9.1f} us/launch  SALU {salu:.2f}  VALU {valu:.2f}  VALU/SALU instr {c.get('SQ_INSTS_VALU',0)/max(1,c.get('SQ_INSTS_SALU',1)):.2f}  wait_inst {c.get('SQ_WAIT_INST_ANY',0)/max(1,c.get('SQ_WAVE_CYCLES',1)):.2f}")
PY
