// init_table_group_config.hpp — see init_table_config.hpp (both helpers live there).
#pragma once
#include <petuum_ps_common/include/init_table_config.hpp>
