import csv, sys, collections
for tag in sys.argv[1:]:
    rows = list(csv.DictReader(open(f'/root/repo/gpurun_out/s2_fa_pmc/{tag}/run_counter_collection.csv')))
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in rows:
        k = r['Kernel_Name']
        if 'fa::' not in k: continue
        k = k.split('fa::')[1].split('(')[0]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        n[(k, r['Counter_Name'])] += 1
    for k, d in agg.items():
        c = n[(k, 'SQ_WAVE_CYCLES')]
        w = d['SQ_WAVE_CYCLES']
        print(f"{tag:4s} {k:40s} waves-cyc {w/c:.3g}  wait_any {d['SQ_WAIT_ANY']/w:.2f} wait_inst {d['SQ_WAIT_INST_ANY']/w:.2f} (lds {d['SQ_WAIT_INST_LDS']/w:.2f}) active {d['SQ_ACTIVE_INST_ANY']/w:.2f} bankconf {d['SQ_LDS_BANK_CONFLICT']/c:.3g} mfma_busy {d['SQ_VALU_MFMA_BUSY_CYCLES']/c:.3g} valu {d['SQ_INSTS_VALU']/c:.3g}")
