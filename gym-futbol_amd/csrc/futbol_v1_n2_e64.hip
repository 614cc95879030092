// futbol_v1_n2_e64.hip -- the envs_v1 kernels for number_of_player = 2 (futbol_v1_inst.hpp)
#include "futbol_v1_inst.hpp"
FUTBOL_V1_INSTANCE(2)
