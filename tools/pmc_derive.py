"""Derived per-kernel ratios from tools/pmc_summarize.py's json (development tool): MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES
over GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs, the round-4 definition), VALU / SALU / LDS instructions per MFMA (SQ_INSTS_VALU
counts the MFMAs too; the ratio here excludes them), wave-cycle shares waiting / issuing, LDS bank-conflict share."""
import json
import sys

d = json.load(open(sys.argv[1]))
for name, c in d.items():
    g = lambda k: c.get(k)  # noqa: E731
    out = {}
    mf = g("SQ_INSTS_MFMA")
    if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        out["mfma_busy"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / (g("GRBM_GUI_ACTIVE") / 8 * 1024)
    if mf:
        if g("SQ_INSTS_VALU") is not None:
            out["valu_per_mfma"] = (g("SQ_INSTS_VALU") - mf) / mf
        for k in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
            if g(k) is not None:
                out[k[9:].lower() + "_per_mfma"] = g(k) / mf
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_MFMA", "SQ_ACTIVE_INST_LDS"):
            if g(k) is not None:
                out[k[3:].lower() + "_frac"] = g(k) / wc
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    if g("GRBM_GUI_ACTIVE"):
        out["gui_active_cycles"] = g("GRBM_GUI_ACTIVE")
    print(name[:100])
    print("   " + ", ".join(f"{k} {v:.3f}" if v < 100 else f"{k} {v:.0f}" for k, v in out.items()))
