// Slotted-kernel launchers, fp32 (U = 16 rows per step; 8 measured slower on FE).
#define VBC_SLOTS_T float
#define VBC_SLOTS_U 16
#define VBC_SLOTS_SUFFIX f32
#include "vbc_slots_launch.inc"
