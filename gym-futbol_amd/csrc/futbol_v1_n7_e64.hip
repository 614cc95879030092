// futbol_v1_n7_e64.hip -- the envs_v1 kernels for number_of_player = 7 (futbol_v1_inst.hpp)
#include "futbol_v1_inst.hpp"
FUTBOL_V1_INSTANCE(7)
