// eegfusion_internal.h — enums shared by the kernels and the C-ABI (mirrors include/eegfusion.h).
#pragma once
#include "../../include/eegfusion.h"

extern int g_ln_rpw;  // layernorm.hip: rows per wave of eegf_ln_fwd (eegf_tune key 6)
extern int g_ln_bwd_rpb;  // layernorm.hip: rows per workgroup of eegf_ln_bwd at rows >= 65536 (eegf_tune key 7)
