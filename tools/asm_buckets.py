"""Dynamic instruction mix of a gfx950 kernel from its assembly listing, bucketed.

    python tools/asm_buckets.py <listing.s> <spec.json> [out.json]

The listing is `hipcc --offload-device-only -S` of the shipped source with the Makefile's flags.  The
spec names the kernel and the execution count of its basic blocks per work unit (one credential: a lane
pair for the pair-lane kernels, a lane quad for the quad fexp), by label; a block without an entry runs as
often as the block before it (fall-through).  Calls are resolved to their callees (s_getpc / s_add_u32
sym@rel32@lo / s_swappc), each callee counted with its own block weights (spec "callees", default 1 per
call for every block), recursively.  Labels are the listing's `.LBBf_b:` lines and its `; %bb.N:`
comments (the fall-through blocks of exec-mask branches): a branch no lane takes skips its blocks
(s_cbranch_execz), so the spec gives them weight 0.

Buckets (per lane, per work unit), following VERDICT r05's list:
  mad           v_mad_u64_u32 / v_mad_i64_i32: the product scans' 32x32->64 multiply-adds
  carry_mderiv  the column carries and the Montgomery m derivation: 64-bit shifts, v_lshl_add_u64, masks,
                alignbit / bfe / perm, add/sub with carry, v_mul_lo/hi
  addsub        carry-free 32-bit limb additions / subtractions (the lazy field's sums)
  exchange      DPP moves (partner halves), selects (v_cndmask), lane exchanges (ds_bpermute, readlane)
  vmov          plain register moves and AGPR <-> VGPR moves
  valu_other    any other vector ALU instruction
  scratch_ld / scratch_st   spills and the callee-saved register saves (scratch memory)
  lds           LDS reads / writes (the parked twist points, packed), not exchanges
  global        global / buffer memory
  salu          scalar ALU and exec-mask manipulation
  branch_call   branches, calls, returns
  nop_wait      s_nop hazard padding and s_waitcnt
"""
import collections
import json
import re
import sys

VALU_BUCKETS = ("mad", "carry_mderiv", "addsub", "exchange", "vmov", "valu_other")
ORDER = VALU_BUCKETS + ("scratch_ld", "scratch_st", "lds", "global", "salu", "branch_call", "nop_wait")

CARRY = re.compile(r"v_(ashrrev_i64|lshrrev_b64|lshlrev_b64|lshl_add_u64|and_b32|and_or_b32|or_b32|xor_b32|"
                   r"alignbit_b32|alignbyte_b32|bfe_u32|bfe_i32|bfi_b32|perm_b32|lshl_or_b32|lshrrev_b32|"
                   r"ashrrev_i32|lshlrev_b32|add_co_u32|addc_co_u32|sub_co_u32|subb_co_u32|subrev_co_u32|"
                   r"subbrev_co_u32|mul_lo_u32|mul_hi_u32|mul_hi_i32|not_b32|lshl_add_u32|add_lshl_u32|"
                   r"or3_b32|and_b64|or_b64|xor_b64|lshrrev_b16|bfrev_b32|ffbh_u32|ffbl_b32|cvt_\w+|rndne_\w+|"
                   r"fma_f64|mul_f64|add_f64|fract_\w+|ldexp_\w+|floor_\w+)")
ADDSUB = re.compile(r"v_(add_u32|sub_u32|subrev_u32|add3_u32|add_i32|sub_i32|add_nc_u32|sub_nc_u32|"
                    r"mad_u32_u24|mad_i32_i24|mul_u32_u24|mul_i32_i24|max_\w+|min_\w+|sad_u32|med3_\w+)")


def bucket(ins, line):
    if ins in ("v_mad_u64_u32", "v_mad_i64_i32"):
        return "mad"
    if ins.startswith("v_"):
        if "_dpp" in ins or "dpp" in line or ins.startswith(("v_cndmask", "v_readlane", "v_writelane",
                                                              "v_readfirstlane", "v_permlane", "v_mov_b32_sdwa")):
            return "exchange"
        if ins.startswith(("v_mov_b32", "v_mov_b64", "v_accvgpr", "v_pk_mov")):
            return "vmov"
        if CARRY.match(ins):
            return "carry_mderiv"
        if ADDSUB.match(ins):
            return "addsub"
        return "valu_other"
    if ins.startswith("scratch_load"):
        return "scratch_ld"
    if ins.startswith("scratch_store"):
        return "scratch_st"
    if ins.startswith(("ds_bpermute", "ds_permute", "ds_swizzle")):
        return "exchange"
    if ins.startswith("ds_"):
        return "lds"
    if ins.startswith(("global_", "buffer_", "flat_")):
        return "global"
    if ins in ("s_nop", "s_waitcnt") or ins.startswith("s_waitcnt"):
        return "nop_wait"
    if ins.startswith(("s_cbranch", "s_branch", "s_swappc", "s_setpc", "s_getpc", "s_endpgm")):
        return "branch_call"
    if ins.startswith("s_"):
        return "salu"
    return "valu_other"


def parse(path):
    """function name -> list of blocks {label, counts (Counter of buckets), calls [callee]}"""
    txt = open(path).read()
    funcs = {}
    for chunk in re.split(r"\n(?=_Z[\w.]+:)", txt):
        name = chunk.split(":", 1)[0].strip()
        if not name.startswith("_Z"):
            continue
        blocks = [{"label": "entry", "counts": collections.Counter(), "calls": [], "ops": collections.Counter()}]
        regsym = {}
        for line in chunk.split("\n")[1:]:
            m = re.match(r"^(\.LBB\d+_\d+):", line) or re.match(r"^; (%bb\.\d+):", line)
            if m:
                blocks.append({"label": m.group(1), "counts": collections.Counter(), "calls": [],
                               "ops": collections.Counter()})
                continue
            if not line.startswith("\t"):
                continue
            s = line.strip()
            if not s or s.startswith((".", ";")):
                continue
            ins = s.split()[0]
            mm = re.match(r"s_add_u32\s+(s\d+),\s*s\d+,\s*([\w.$]+)@rel32@lo", s)
            if mm:
                regsym[mm.group(1)] = mm.group(2)
            if ins == "s_swappc_b64":
                r = re.search(r"s\[(\d+):\d+\]\s*$", s)
                blocks[-1]["calls"].append(regsym.get("s" + r.group(1), "?") if r else "?")
            blocks[-1]["counts"][bucket(ins, s)] += 1
            blocks[-1]["ops"][ins] += 1
        funcs[name] = blocks
    return funcs


def short(name):
    m = re.search(r"L?\d+([a-z_0-9]+?)E", name)
    for key in ("k_miller", "k_fexp_q", "miller_add", "q_pow_x_gs", "lz_f2_mul_call", "lz_f2_sqr_call", "lz_mul_call",
                "lz_canon_call", "f2_mul_call", "fp_mul_call", "t_check", "k_prep", "k_msm_straus"):
        if key in name:
            return key
    return m.group(1) if m else name[:40]


def dyn(funcs, fname, weights, spec_callees, memo, depth=0):
    """dynamic bucket counts of one execution of fname with block weights `weights`"""
    key = (fname, json.dumps(weights, sort_keys=True))
    if key in memo:
        return memo[key]
    tot = collections.Counter()
    own = collections.Counter()
    calls = collections.Counter()
    ops = collections.Counter()
    w = 1.0
    for b in funcs[fname]:
        w = weights.get(b["label"], w)
        for k, v in b["counts"].items():
            own[k] += w * v
        for k, v in b["ops"].items():
            ops[k] += w * v
        for c in b["calls"]:
            calls[c] += w
    tot.update(own)
    per_callee = {}
    for c, k in calls.items():
        if c not in funcs:
            continue
        sub = dyn(funcs, c, spec_callees.get(short(c), {}), spec_callees, memo, depth + 1)
        per_callee[c] = {"calls": k, "per_call": sub["total"]}
        for b, v in sub["total"].items():
            tot[b] += k * v
    r = {"total": tot, "own": own, "calls": per_callee, "own_ops": ops}
    memo[key] = r
    return r


def region(funcs, fname, weights, labels, spec_callees):
    """dynamic bucket counts of the blocks `labels` of fname (their own instructions and their calls)"""
    tot = collections.Counter()
    w = 1.0
    for b in funcs[fname]:
        w = weights.get(b["label"], w)
        if b["label"] not in labels:
            continue
        for k, v in b["counts"].items():
            tot[k] += w * v
        for c in b["calls"]:
            if c in funcs:
                sub = dyn(funcs, c, spec_callees.get(short(c), {}), spec_callees, {})
                for k2, v2 in sub["total"].items():
                    tot[k2] += w * v2
    return tot


def summarize(c, alg_mads=None, pmc_valu=None):
    valu = sum(c.get(b, 0) for b in VALU_BUCKETS)
    out = {b: round(c.get(b, 0)) for b in ORDER}
    out["valu"] = round(valu)
    out["all"] = round(sum(c.values()))
    if alg_mads:
        out["valu_per_alg_mad"] = round(valu / alg_mads, 3)
        out["share_of_valu"] = {b: round(c.get(b, 0) / valu, 4) for b in VALU_BUCKETS}
    if pmc_valu:
        out["pmc_valu_per_unit"] = round(pmc_valu)
        out["model_over_pmc"] = round(valu / pmc_valu, 3)
    return out


def main():
    lst, specf = sys.argv[1], sys.argv[2]
    spec = json.load(open(specf))
    funcs = parse(lst)
    kern = [f for f in funcs if spec["kernel"] in f]
    assert len(kern) == 1, (spec["kernel"], kern)
    kern = kern[0]
    r = dyn(funcs, kern, spec["blocks"], spec.get("callees", {}), {})
    lanes = spec.get("lanes_per_unit", 1)
    alg = spec.get("algorithmic_mads_per_unit")
    alg_lane = alg / lanes if alg else None
    res = {
        "listing": spec.get("listing", lst), "kernel": kern, "unit": spec.get("unit"),
        "lanes_per_unit": lanes, "algorithmic_mads_per_unit": alg,
        "note": "per LANE per work unit (dynamic: block weights x static counts, calls expanded); "
                "valu_per_alg_mad = VALU lane-ops / algorithmic mads of that lane's share",
        "total": summarize(r["total"], alg_lane, spec.get("pmc_valu_per_lane")),
        "kernel_own": summarize(r["own"], alg_lane),
        "callees": {short(c): {"calls_per_unit": round(v["calls"], 2), "per_call": summarize(v["per_call"])}
                    for c, v in sorted(r["calls"].items(), key=lambda kv: -kv[1]["calls"])},
        "kernel_own_top_ops": {k: round(v) for k, v in r["own_ops"].most_common(25)},
    }
    if spec.get("regions"):
        res["regions"] = {}
        for name, labels in spec["regions"].items():
            c = region(funcs, kern, spec["blocks"], set(labels), spec.get("callees", {}))
            sm = summarize(c)
            sm["share_of_total_valu"] = round(sm["valu"] / res["total"]["valu"], 4)
            sm["non_mad_share_of_region_valu"] = round(1 - sm["mad"] / max(sm["valu"], 1), 4)
            res["regions"][name] = sm
    for c, v in r["calls"].items():
        res["callees"][short(c)]["share_of_total_valu"] = round(
            v["calls"] * sum(v["per_call"].get(b, 0) for b in VALU_BUCKETS) / res["total"]["valu"], 4)
    js = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
