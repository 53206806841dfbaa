#!/usr/bin/env python3
"""Issue-rate tables for profiles/valu_rates_r02.md from the microbenchmark
outputs (tools/valu_rates.hip, salsa_mix.hip, dep_mix.hip, vgpr_banks.py,
vmem_issue.hip, lds_ua_rate.hip), plus the roofline.valu peak bench.py uses.

Usage: tools/valu_table.py DIR > profiles/valu_rates_r02.md
(DIR holds valu_rates.jsonl, salsa_mix.jsonl, dep_mix.jsonl, vgpr_banks.jsonl,
vmem_issue.txt, lds_ua_rate.jsonl as the tools print them)."""
import collections
import json
import os
import sys


def rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip().startswith("{")]


def table(recs, title, unit):
    by = collections.OrderedDict()
    waves = set()
    for r in recs:
        if "cycles_per_unit_per_simd" not in r:
            continue
        by.setdefault(r["op"], {})[r["waves_per_simd"]] = r["cycles_per_unit_per_simd"]
        waves.add(r["waves_per_simd"])
    if not by:
        return ""
    ws = sorted(waves)
    out = [f"### {title}", "", f"{unit} per SIMD, by waves per SIMD:", "",
           "| op | " + " | ".join(f"{w} w" for w in ws) + " |",
           "|---|" + "---:|" * len(ws)]
    for op, d in by.items():
        out.append(f"| `{op}` | " + " | ".join(f"{d[w]:.2f}" if w in d else "" for w in ws) + " |")
    return "\n".join(out) + "\n"


def main():
    d = sys.argv[1]
    vr = rows(os.path.join(d, "valu_rates.jsonl"))
    print("# gfx950 issue rates (round 2)\n")
    print("Measured on one MI355X (256 CUs) with the tools named in each section;")
    print("cycles = kernel wall time x the in-kernel shader clock (s_memtime over")
    print("s_memrealtime), per SIMD.  At 1 wave per SIMD every VALU instruction")
    print("costs at least 4 cycles (one quad-cycle, PMC `SQ_ACTIVE_INST_VALU`), and the")
    print("1-wave column includes loop and clock-read overhead the other columns amortise.\n")
    print(table(vr, "VALU instructions (tools/valu_rates.hip)", "cycles per wave64 instruction"))
    print(table(rows(os.path.join(d, "salsa_mix.jsonl")),
                "Salsa20 block encodings (tools/salsa_mix.hip)", "cycles per block (or per instruction for mixes)"))
    print(table(rows(os.path.join(d, "dep_mix.jsonl")),
                "Dependent add->alignbit->xor chains (tools/dep_mix.hip)", "cycles per instruction"))
    print(table(rows(os.path.join(d, "vgpr_banks.jsonl")),
                "VGPR bank probes (tools/vgpr_banks.py)", "cycles per instruction"))
    vm = os.path.join(d, "vmem_issue.txt")
    if os.path.exists(vm):
        print("### Global dwordx4 issue cost by access shape (tools/vmem_issue.hip)\n")
        print("One wave per SIMD; each instruction's 64 lanes spread over 64/LPP")
        print("pieces of 64 bytes strided 1,057 bytes apart (the config-2 frame")
        print("stride); a4 = 4-byte aligned, a16 = 16-byte aligned.\n")
        print("```")
        print(open(vm).read().rstrip())
        print("```\n")
    lu = rows(os.path.join(d, "lds_ua_rate.jsonl"))
    if lu:
        bad = sum(r.get("bad_bits", 0) for r in lu if "check" in r)
        print(table(lu, "LDS access, aligned vs unaligned (tools/lds_ua_rate.hip)", "cycles per wave-instruction"))
        print(f"Unaligned ds_read/ds_write correctness checks: {sum(1 for r in lu if 'check' in r)} offsets, "
              f"{bad} wrong bits.\n")
    # the peak bench.py reports as roofline.valu.peak
    best = {}
    for r in vr:
        if r["op"] in ("v_add_u32", "v_xor_b32") and "cycles_per_unit_per_simd" in r:
            best[r["waves_per_simd"]] = min(best.get(r["waves_per_simd"], 1e9), r["cycles_per_unit_per_simd"])
    if best:
        c = min(best.values())
        print("### roofline.valu.peak\n")
        print(f"Fastest VOP2 integer issue measured: {c:.2f} cycles per wave64 instruction per SIMD")
        print(f"= {64 / c:.1f} lane-operations per cycle per SIMD.  bench.py prices the frame")
        print("kernel's VALU work against that rate x 1,024 SIMDs x the kernel's measured")
        print("shader clock; the Salsa20 block itself issues at ~4 cycles per instruction")
        print("at every occupancy (table above), so the Salsa-bound ceiling is ~0.6 of it.")


if __name__ == "__main__":
    main()
