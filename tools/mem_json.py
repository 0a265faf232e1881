#!/usr/bin/env python3
"""gpurun_out/mem_<tag>.txt (tools/mem_passes.sh: one `enc {...}` and one `dec {...}` line of
pass-prefixed counters) -> the memory-pipeline JSON under profiles/ (DIAGNOSTIC).

Derivation: GRBM_GUI_ACTIVE (in every pass, averaged) is summed over the 8 XCDs, so the kernel
runs cycles_per_xcd = GUI_ACTIVE / 8; TA / TD / TCP counters are summed over the 256 CUs and TCC
over the 128 L2 channels, so busy fractions = counter / (units x cycles_per_xcd).
usage: mem_json.py gpurun_out/mem_<tag>.txt NBLOCKS NOTE > profiles/<name>.json"""
import ast
import json
import sys


def derive(raw, nb):
    c, gui = {}, []
    for k, v in raw.items():
        name = k.split(":", 1)[1]
        if name == "GRBM_GUI_ACTIVE":
            gui.append(float(v))
        else:
            c[name] = float(v)
    cyc = sum(gui) / len(gui) / 8.0
    cu, ch = 256.0 * cyc, 128.0 * cyc
    return {
        "counters": c,
        "cycles_per_xcd": round(cyc),
        "TA_busy_frac": round(c["TA_TA_BUSY"] / cu, 3),
        "TD_busy_frac": round(c["TD_TD_BUSY"] / cu, 3),
        "TCC_busy_frac": round(c["TCC_BUSY"] / ch, 3),
        "TD_stalled_on_TC_frac": round(c["TD_TC_STALL"] / cu, 3),
        "TA_addr_stalled_on_TC_frac": round(c["TA_ADDR_STALLED_BY_TC_CYCLES"] / cu, 3),
        "L2_hit_rate": round(c["TCC_HIT"] / (c["TCC_HIT"] + c["TCC_MISS"]), 3),
        "L1_to_L2_reads_per_block": round(c["TCP_TCC_READ_REQ"] / nb, 1),
    }


def main():
    path, nb, note = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    out = {"_note": note}
    for line in open(path):
        kind, _, rest = line.partition(" ")
        if kind in ("enc", "dec"):
            out["lz4_encode_kernel" if kind == "enc" else "lz4_decode_kernel"] = derive(
                ast.literal_eval(rest.strip()), nb)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
