"""Generates pqh_heap_asm.h: the register-heap sifts of huff_trees_wave (pqh_tables.hip) as
gfx950 inline asm.  One wavefront per tree; heap slot s lives in VGPR v(40 + ((s + 1) >> 6))
at lane (s + 1) & 63 (v40: slots 0..62, v41: 63..126, v42: 127..190, v43: 191..254, v44:
slot 255 at lane 0 -- every other lane of v44 and of v45..v47 is a sentinel); keys are
u32 weight << 10 | tie << 9 | node, the sentinel 0xFFFFFFFF.  The sifts are unrolled by
depth, so every access names its register statically: a heap read is one v_readlane with
a scalar lane index, a write one v_writelane, the control state (slot index, keys) stays in
SGPRs.  Reference semantics (huffman_encode.c:33-76): push sifts up while strictly lighter
than the parent; pop moves the last entry down from the root, taking the left child unless
the right one is strictly lighter, while strictly heavier than that child.

Run: python pq_huffman_amd/csrc/gen/heap_asm.py > pq_huffman_amd/csrc/hip/pqh_heap_asm.h
"""

TIE, NOTIE, WMASK = "0x200", "0xfffffdff", "0xfffffc00"


def reg_access(depth, slot1, lab, body):
    """Code that runs `body(vreg, lane_sgpr)` for the slot whose (s + 1) is in SGPR slot1
    (clobbered: it becomes the lane) at the given depth; depth 7 branches on the register."""
    if depth <= 5:
        return body("v40", slot1)
    if depth == 6:
        return [f"s_sub_u32 {slot1}, {slot1}, 64"] + body("v41", slot1)
    if depth == 7:
        out = [f"s_cmp_lt_u32 {slot1}, 192", f"s_cbranch_scc0 {lab}_h",
               f"s_sub_u32 {slot1}, {slot1}, 128"] + body("v42", slot1) + \
              [f"s_branch {lab}_j", f"{lab}_h:", f"s_sub_u32 {slot1}, {slot1}, 192"] + \
              body("v43", slot1) + [f"{lab}_j:"]
        return out
    return body("v44", "0")            # depth 8: slot 255 only


def wl(v, val, ln):
    """v_writelane with an SGPR value: the lane select must be M0 (one constant-bus read)."""
    return [f"s_mov_b32 m0, {ln}", "s_nop 0", f"v_writelane_b32 {v}, {val}, m0"]


def gen_pop():
    # in: %[sz] = size after the decrement; out: %[top]
    # scratch SGPRs: i c ln kl kr kc lw last t
    L = []
    L += ["s_nop 4", "s_mov_b32 %[m0s], m0",
          "v_readlane_b32 %[top], v40, 1",                      # slot 0
          # last = slot sz; its slot becomes a sentinel
          "s_add_u32 %[c], %[sz], 1"]
    # the last slot can be at any depth: dispatch on (sz + 1) >> 6 (its register)
    L += ["s_lshr_b32 %[t], %[c], 6", "s_and_b32 %[ln], %[c], 63",
          "s_cmp_eq_u32 %[t], 0", "s_cbranch_scc0 .Lpl1_%=",
          "v_readlane_b32 %[last], v40, %[ln]", "v_writelane_b32 v40, -1, %[ln]", "s_branch .Lpld_%=",
          ".Lpl1_%=:", "s_cmp_eq_u32 %[t], 1", "s_cbranch_scc0 .Lpl2_%=",
          "v_readlane_b32 %[last], v41, %[ln]", "v_writelane_b32 v41, -1, %[ln]", "s_branch .Lpld_%=",
          ".Lpl2_%=:", "s_cmp_eq_u32 %[t], 2", "s_cbranch_scc0 .Lpl3_%=",
          "v_readlane_b32 %[last], v42, %[ln]", "v_writelane_b32 v42, -1, %[ln]", "s_branch .Lpld_%=",
          ".Lpl3_%=:", "s_cmp_eq_u32 %[t], 3", "s_cbranch_scc0 .Lpl4_%=",
          "v_readlane_b32 %[last], v43, %[ln]", "v_writelane_b32 v43, -1, %[ln]", "s_branch .Lpld_%=",
          ".Lpl4_%=:",
          "v_readlane_b32 %[last], v44, 0", "v_writelane_b32 v44, -1, 0",
          ".Lpld_%=:",
          "s_and_b32 %[lw], %[last], " + WMASK,
          "s_mov_b32 %[i], 0",
          "s_cmp_eq_u32 %[sz], 0", "s_cbranch_scc1 .Lpend_%="]   # popped the only entry
    for d in range(8):                                          # parent at depth d
        lab = f".Lpd{d}_%="
        L += [f"s_lshl_b32 %[c], %[i], 1", f"s_add_u32 %[ln], %[c], 2"]   # (left child) + 1
        if d + 1 <= 7:
            L += reg_access(d + 1, "%[ln]", lab + "r",
                            lambda v, ln: [f"v_readlane_b32 %[kl], {v}, {ln}",
                                           f"s_add_u32 {ln}, {ln}, 1",
                                           f"v_readlane_b32 %[kr], {v}, {ln}"])
        else:                                                   # children at depth 8
            L += ["s_mov_b32 %[kl], -1", "s_cmp_eq_u32 %[i], 127", f"s_cbranch_scc0 {lab}n",
                  "v_readlane_b32 %[kl], v44, 0", f"{lab}n:", "s_mov_b32 %[kr], -1"]
        L += ["s_or_b32 %[kr], %[kr], " + TIE, "s_min_u32 %[kc], %[kl], %[kr]",
              "s_cmp_lt_u32 %[kc], %[lw]", f"s_cbranch_scc0 .Lpput{d}_%="]
        # slot i = the child (its tie bit cleared)
        L += ["s_and_b32 %[kl], %[kc], " + NOTIE, "s_add_u32 %[t], %[i], 1"]
        L += reg_access(d, "%[t]", lab + "w", lambda v, ln: wl(v, "%[kl]", ln))
        L += ["s_bfe_u32 %[kr], %[kc], 0x10009", "s_add_u32 %[i], %[c], 1",
              "s_add_u32 %[i], %[i], %[kr]"]
    L += ["s_add_u32 %[t], %[i], 1"]                            # place at depth 8 (slot 255)
    L += reg_access(8, "%[t]", ".Lpd8w_%=", lambda v, ln: wl(v, "%[last]", ln))
    L += ["s_branch .Lpend_%="]
    for d in range(8):
        L += [f".Lpput{d}_%=:", "s_add_u32 %[t], %[i], 1"]
        L += reg_access(d, "%[t]", f".Lpp{d}w_%=",
                        lambda v, ln: wl(v, "%[last]", ln))
        L += ["s_branch .Lpend_%="]
    L += [".Lpend_%=:", "s_mov_b32 m0, %[m0s]", "s_nop 4"]
    return L


def gen_push():
    # in: %[i] = slot (size before the increment), %[e] = key; scratch: p ln hp hw t d
    L = ["s_nop 4", "s_mov_b32 %[m0s], m0",
         "s_add_u32 %[t], %[i], 1", "s_flbit_i32_b32 %[d], %[t]",   # leading zeros of i + 1
         "s_sub_u32 %[d], 31, %[d]"]                                  # depth of slot i
    for D in range(8, 0, -1):
        L += [f"s_cmp_eq_u32 %[d], {D}", f"s_cbranch_scc1 .Lu{D}_%="]
    L += ["s_branch .Luput0_%="]
    for D in range(8, 0, -1):
        lab = f".Lu{D}_%="
        L += [f"{lab}:",
              "s_add_u32 %[p], %[i], -1", "s_lshr_b32 %[p], %[p], 1",   # parent (depth D - 1)
              "s_add_u32 %[ln], %[p], 1"]
        L += reg_access(D - 1, "%[ln]", lab + "r", lambda v, ln: [f"v_readlane_b32 %[hp], {v}, {ln}"])
        L += ["s_and_b32 %[hw], %[hp], " + WMASK, "s_cmp_lt_u32 %[e], %[hw]",
              f"s_cbranch_scc0 .Luput{D}_%="]
        L += ["s_add_u32 %[t], %[i], 1"]                        # slot i = the parent
        L += reg_access(D, "%[t]", lab + "w", lambda v, ln: wl(v, "%[hp]", ln))
        L += ["s_mov_b32 %[i], %[p]"]                           # falls through to depth D - 1
    L += ["s_branch .Luput0_%="]
    for D in range(8, -1, -1):
        L += [f".Luput{D}_%=:", "s_add_u32 %[t], %[i], 1"]
        L += reg_access(D, "%[t]", f".Lup{D}w_%=", lambda v, ln: wl(v, "%[e]", ln))
        L += ["s_branch .Luend_%="]
    L += [".Luend_%=:", "s_mov_b32 m0, %[m0s]", "s_nop 4"]
    return L


def emit(name, lines):
    body = "\\n\\t".join(lines)
    return f'#define {name} "{body}"\n'


if __name__ == "__main__":
    print("// Generated by pq_huffman_amd/csrc/gen/heap_asm.py -- do not edit.")
    print("#pragma once")
    print(emit("PQH_HEAP_POP_ASM", gen_pop()))
    print(emit("PQH_HEAP_PUSH_ASM", gen_push()))
