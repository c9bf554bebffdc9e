/*
 * oracle/orc_batch.c -- TEST INFRASTRUCTURE ONLY.
 * pthread driver over orc_tdec_run: the "port" CPU baseline when oracle/_ref is not available.
 */
#include <pthread.h>
#include <stdlib.h>

#include "oracle.h"

struct job {
  const int16_t* bufs;
  uint32_t       stride, first, count, K, nhalf;
  uint8_t*       out;
};

static void* worker(void* arg)
{
  struct job* j = arg;
  for (uint32_t i = 0; i < j->count; i++) {
    uint32_t cb = j->first + i;
    orc_tdec_run(&j->bufs[(size_t)cb * j->stride], j->K, j->nhalf, &j->out[(size_t)cb * (j->K / 8)], NULL, NULL);
  }
  return NULL;
}

int orc_tdec_run_batch(const int16_t* bufs, uint32_t stride, uint32_t ncb, uint32_t K, uint32_t nhalf, uint8_t* out,
                       int nthreads)
{
  if (nthreads < 1) nthreads = 1;
  pthread_t*  th   = calloc(nthreads, sizeof(pthread_t));
  struct job* jobs = calloc(nthreads, sizeof(struct job));
  uint32_t    base = ncb / nthreads, rem = ncb % nthreads, first = 0;
  for (int t = 0; t < nthreads; t++) {
    uint32_t c = base + ((uint32_t)t < rem);
    jobs[t]    = (struct job){bufs, stride, first, c, K, nhalf, out};
    first += c;
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
