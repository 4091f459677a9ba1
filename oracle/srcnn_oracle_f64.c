/*
 * srcnn_oracle_f64.c -- the oracle's restatement (srcnn_oracle.c) compiled
 * with double arithmetic: the same loop nests, layouts and quirks, every
 * float of them a double.  TEST INFRASTRUCTURE ONLY (see srcnn_oracle.h).
 *
 * It is the exact-arithmetic yardstick of the parity tests: tests/hip_util.py
 * measures how far the fp32 oracle (the reference's own accumulation order)
 * and the HIP path each land from it, element by element, so that elements
 * whose sums cancel are judged against the error the reference algorithm
 * itself makes there.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define float double
#define fmaxf fmax
#define fminf fmin
#include "srcnn_oracle.c"
