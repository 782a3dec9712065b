// init_table_group_config.hpp — InitTableGroupConfig (src/petuum_ps_common/include/
// init_table_group_config.hpp of the reference): fills a TableGroupConfig from the system
// flags (system_gflags_declare.hpp), as init_table_group_config.cpp:5-55 does.  Defined in
// libpetuum_ps.so (parameter_server_amd/csrc/petuum_flags.cpp).
#pragma once
#include <petuum_ps_common/include/configs.hpp>

namespace petuum {
void InitTableGroupConfig(TableGroupConfig *config, int32_t num_tables);
}  // namespace petuum
