"""Print SQ counter ratios per kernel from a pmcsum JSON: python tools/pmcshow.py FILE [substr]"""
import json, sys
d = json.load(open(sys.argv[1]))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
print(f"{'kernel':34s} {'gui_cyc':>9s} {'wait':>5s} {'winst':>5s} {'act':>5s} {'mfmaU':>5s} {'valu/w':>7s} {'lds/w':>6s} {'vmem/w':>6s} {'salu/w':>6s} {'actVALU':>7s} {'bankc':>8s}")
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
    if 'SQ_WAVE_CYCLES' not in v or sub not in k:
        continue
    w = v['SQ_WAVE_CYCLES']
    gui = v.get('GRBM_GUI_ACTIVE', 0) / 8
    waves = w * 4 / max(gui, 1)   # average resident waves (quad-cycles → cycles)
    mu = v['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / max(gui, 1)
    print(f"{k[:34]:34s} {gui:9.3e} {v['SQ_WAIT_ANY']/w:5.2f} {v['SQ_WAIT_INST_ANY']/w:5.2f} {v['SQ_ACTIVE_INST_ANY']/w:5.2f} {mu:5.2f} "
          f"{v['SQ_INSTS_VALU']/waves:7.0f} {v['SQ_INSTS_LDS']/waves:6.0f} {v.get('SQ_INSTS_VMEM_RD',0)/waves:6.0f} {v.get('SQ_INSTS_SALU',0)/waves:6.0f} "
          f"{v.get('SQ_ACTIVE_INST_VALU',0)*4/max(gui,1)/waves:7.2f} {v.get('SQ_LDS_BANK_CONFLICT',0):8.2e}")
