# round-6 A/B, hot kernel, cost only (results identical: the added
# instructions write dead registers): what one more instruction per YUYV word
# of the fast path costs, by class -- the price of each op the fast path could
# lose.
#  p_vop2   + one v_and_b32_e32 per word (VOP2, the 2.5-cycle class)
#  p_vop3   + one v_add3_u32 per word (3-operand VOP3)
#  p_vopc   + one v_cmp_gt_u32_sdwa into VCC per word (a compare)
FILE = "trik_hsv_chroma.hip"
_AT = "          asm volatile(\"\" : \"+s\"(bal));\n"
def _add(asm):
    return [(_AT, _AT + "          { uint32_t t_ = cw[i]; " + asm + " }\n")]
VARIANTS = {
    "r6m_base": [("kMaxBlock = 1024;", "kMaxBlock = 1024;")],
    "p_vop2": _add("asm volatile(\"v_and_b32_e32 %0, 0xff, %0\" : \"+v\"(t_));"),
    "p_vop3": _add("asm volatile(\"v_add3_u32 %0, %0, %1, %2\" : \"+v\"(t_) : \"v\"(d[i]), \"v\"(cut[i]));"),
    "p_vopc": _add("asm volatile(\"v_cmp_gt_u32_sdwa vcc, %0, %1 src0_sel:BYTE_0 src1_sel:BYTE_2\" :: \"v\"(t_), \"v\"(d[i]) : \"vcc\");"),
}
