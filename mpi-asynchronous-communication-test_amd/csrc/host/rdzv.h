#ifndef XG_RDZV_H
#define XG_RDZV_H
#include <stddef.h>
#include "xg.h"
/* Fills uid (rank 0 creates it) and the file path (rank 0 unlinks it after xg_init). */
int xg_rendezvous(int rank, int nranks, unsigned char uid[XG_UNIQUE_ID_BYTES], char *path, size_t pathlen);
int xg_env_int(const char *a, const char *b, int dflt);
#endif
