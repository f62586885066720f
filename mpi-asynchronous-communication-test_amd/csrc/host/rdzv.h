#ifndef XG_RDZV_H
#define XG_RDZV_H
#include <stddef.h>
#include "xg.h"
/* Fills uid (rank 0 creates it) and the file path (rank 0 unlinks it after xg_init). */
int xg_rendezvous(int rank, int nranks, unsigned char uid[XG_UNIQUE_ID_BYTES], char *path, size_t pathlen);
int xg_env_int(const char *a, const char *b, int dflt);
/* No launcher (no RANK / WORLD_SIZE / PMI_RANK / PMI_SIZE in the environment) and
 * ngpus > 1: this process becomes the parent of an ngpus-process job -- it never
 * touches the GPU, starts ngpus copies of argv (posix_spawn, one per GPU, with RANK,
 * LOCAL_RANK, WORLD_SIZE and one XG_RDZV_KEY set), waits, stops the others when one
 * fails, and returns the highest child exit code (the caller exits with it).
 * Returns -1 when this process is a rank itself (launcher present, or ngpus <= 1). */
int xg_spawn_ranks(int ngpus, char **argv);
#endif
