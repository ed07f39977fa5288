// wmi_persist_q5.hip — the persistent decoder's q5_1 instances
// (k_dec_persist<NS, BT, false, true>: phases A, C, G2, H, I stream the
// layers' q5_1 repacks and dequantise in registers), in a translation unit of
// their own so the build compiles them beside the f16 ones.
#define WMI_PERSIST_Q5_TU
#include "wmi_persist.hip"
