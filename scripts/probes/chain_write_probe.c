/* Chain-text writer throughput probe: gt_par_write over a .chain file,
 * three runs (MMAPTH=1: malloc mmap threshold raised).  Build: see
 * scripts/gpu_write_probe.sh. */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include "gac_tool.h"
static double now(void){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+1e-9*t.tv_nsec;}
static gt_chains C;
static void fn(FILE *f, int64_t i, void *a){(void)a; gt_write_chain(f,&C,i,C.score[i],C.id[i]);}
#include <malloc.h>
int main(int argc,char**argv){ if(getenv("MMAPTH")){mallopt(M_MMAP_THRESHOLD, 1<<30); mallopt(M_TRIM_THRESHOLD, 1<<30);}
  gt_read_chains(argv[1],&C,-1e300,1);
  for(int k=0;k<3;k++){
    FILE*o=fopen(argv[2],"w"); double t=now(); gt_par_write(o,C.n,fn,NULL); fclose(o); printf("write %.3f s\n",now()-t);}
  return 0;}
