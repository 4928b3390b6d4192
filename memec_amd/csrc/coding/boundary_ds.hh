// boundary_ds.hh — ChunkUtil / TempChunkPool for the adapter's .cc files.
// Inside a MemEC tree these come from common/ds (chunk_util.hh:13-387,
// chunk_pool.hh:38-53), which include coding/coding.hh themselves, so they
// cannot be pulled in by coding.hh; standalone, boundary.hh has them.
#ifndef MEMEC_AMD_CODING_BOUNDARY_DS_HH
#define MEMEC_AMD_CODING_BOUNDARY_DS_HH

#include "coding.hh"

#ifdef MEMEC_TREE
#include "../ds/chunk_pool.hh"
#include "../ds/chunk_util.hh"
#endif

#endif
