// Library identification for the C ABI (include/vggt_mi355x.h).
#include "../../include/vggt_mi355x.h"

extern "C" const char* vggt_version(void) { return "vggt_mi355x 0.1 gfx950"; }
