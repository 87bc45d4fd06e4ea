// Slotted-kernel launchers, fp64 (U = 8 rows per step; 4 measured 4-8 % slower on FE).
#define VBC_SLOTS_T double
#define VBC_SLOTS_U 8
#define VBC_SLOTS_SUFFIX f64
#include "vbc_slots_launch.inc"
