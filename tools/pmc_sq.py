"""MFMA-busy fraction, held clock and wait share of the dominant screen instance from a
tools/pmc_summary.py summary of one SQ/GRBM pass over bench.py (tools/gpu.sh pmc), as JSON
for bench.py's roofline (counter normalisation as MI355X_MICROARCH.md: GRBM_GUI_ACTIVE
sums 8 XCDs, SQ_VALU_MFMA_BUSY_CYCLES sums 1024 SIMDs).

    python tools/pmc_sq.py summary.txt [kernel-substring]"""
import json
import re
import sys

from pmc_traffic import screen_src_sha1


def parse(path):
    blocks, cur = {}, None
    for line in open(path):
        m = re.match(r'^(\S.*?)  dispatches (\d+)  mean duration ([\d.]+) us', line)
        if m:
            cur = m.group(1)
            blocks[cur] = {'dispatches': int(m.group(2)), 'us': float(m.group(3))}
        elif cur and line.strip():
            k, v = line.split()
            blocks[cur][k] = float(v)
    return blocks


def main(path, sub=None):
    b = parse(path)
    subs = [sub] if sub else ['k_screen16rILi11E', 'k_screen16pILi11E', 'k_screen16iILi11E']
    name = next(k for s in subs for k in b if s in k)
    d = b[name]
    cyc = d['GRBM_GUI_ACTIVE'] / 8
    out = {'kernel': name, 'dispatches': d['dispatches'], 'mean_us': d['us'],
           'clock_ghz': cyc / (d['us'] * 1e3),
           'mfma_busy': d['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc,
           'wait_inst_share': d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES'],
           # conflict cycles over LDS-active cycles (SQ_LDS_IDX_ACTIVE); round 5 divided by
           # SQ_ACTIVE_INST_LDS, an instruction count, and overstated the share (0.357 vs 0.105)
           'lds_bank_conflict_share': (d['SQ_LDS_BANK_CONFLICT'] / d['SQ_LDS_IDX_ACTIVE']
                                       if 'SQ_LDS_BANK_CONFLICT' in d and 'SQ_LDS_IDX_ACTIVE' in d else None),
           'wait_any_share': d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES'] if 'SQ_WAIT_ANY' in d else None,
           'mfma_coexec': (d['SQ_VALU_MFMA_COEXEC_CYCLES'] / 1024 / cyc
                           if 'SQ_VALU_MFMA_COEXEC_CYCLES' in d else None),
           'screen_src_sha1': screen_src_sha1(),
           'note': 'one rocprofv3 --pmc pass over bench.py (GRBM_GUI_ACTIVE / 8 = cycles, '
                   'SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / cycles = MFMA busy)'}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:3])
