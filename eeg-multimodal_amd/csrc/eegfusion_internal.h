// eegfusion_internal.h — enums shared by the kernels and the C-ABI (mirrors include/eegfusion.h).
#pragma once
#include "../../include/eegfusion.h"
