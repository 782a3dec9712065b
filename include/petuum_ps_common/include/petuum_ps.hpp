// petuum_ps.hpp — what apps include (src/petuum_ps_common/include/petuum_ps.hpp:1-15).
#pragma once

// (the reference's petuum_ps.hpp reaches <cassert> through multiplicative_dense_row.hpp, and
// apps call assert without including it: apps/lda/src/lda_engine.cpp:315)
#include <cassert>

#include <petuum_ps_common/include/configs.hpp>
#include <petuum_ps_common/include/init_table_config.hpp>
#include <petuum_ps_common/include/init_table_group_config.hpp>
#include <petuum_ps_common/include/ps_table_group.hpp>
#include <petuum_ps_common/include/table.hpp>
#include <petuum_ps_common/storage/dense_row.hpp>
#include <petuum_ps_common/storage/dense_row_float16.hpp>
#include <petuum_ps_common/storage/sorted_vector_map_row.hpp>
#include <petuum_ps_common/storage/sparse_row.hpp>
#include <petuum_ps_common/util/utils.hpp>
#include <petuum_ps_common/util/stats.hpp>
#include <petuum_ps_common/util/high_resolution_timer.hpp>
