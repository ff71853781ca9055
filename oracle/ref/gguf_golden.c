// Golden vectors for the GGUF Q4_0 x Q8_0 path from the reference's own code: neural_speed/core/data_types.h,
// neural_speed/vectors/cpu/quantize.h and neural_speed/core/layers/vec_dot.h, compiled here as C for the host's
// baseline ISA (their scalar paths).  The fp16 -> fp32 lookup table is filled by the loop ne_init runs
// (ne_layers.c:738-742).  Test infrastructure only (oracle/ref/Makefile -> oracle/_ref/gguf_golden).
#include <float.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "core/data_types.h"
#include "vectors/cpu/quantize.h"
#include "core/layers/vec_dot.h"

static const char* g_dir;
static FILE* g_man;

static void dump(const char* cs, const char* name, const char* dt, const void* p, size_t esz, size_t n) {
  char path[1024];
  snprintf(path, sizeof(path), "%s/%s.%s.bin", g_dir, cs, name);
  FILE* f = fopen(path, "wb");
  fwrite(p, esz, n, f);
  fclose(f);
  fprintf(g_man, "%s %s %s %zu\n", cs, name, dt, n);
}

static uint32_t g_state = 20250113u;
static uint32_t rnd(void) {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 17;
  g_state ^= g_state << 5;
  return g_state;
}
static float urand(float lo, float hi) { return lo + (hi - lo) * (float)(rnd() & 0xFFFFFF) / 16777216.f; }

static void case_q4_0(const char* cs, int n, int k, int m, float amp) {
  float* W = malloc(sizeof(float) * n * k);
  for (int i = 0; i < n * k; i++) W[i] = urand(-amp, amp);
  for (int j = 0; j < k && n > 1; j++) W[k + j] = 0.f;     // row 1: all zero (d = 0)
  if (n > 2) W[2 * k + 5] = 40.f * amp;                    // row 2: one outlier per row
  const int nb = k / QK4_0;
  block_q4_0* Q = malloc(sizeof(block_q4_0) * n * nb);
  float* D = malloc(sizeof(float) * n * k);
  for (int r = 0; r < n; r++) {
    quantize_row_q4_0(W + (size_t)r * k, Q + (size_t)r * nb, k);
    dequantize_row_q4_0(Q + (size_t)r * nb, D + (size_t)r * k, k);
  }
  float* A = malloc(sizeof(float) * m * k);
  for (int i = 0; i < m * k; i++) A[i] = urand(-1.f, 1.f);
  block_q8_0* Y = malloc(sizeof(block_q8_0) * m * nb);
  float* C = malloc(sizeof(float) * m * n);
  for (int i = 0; i < m; i++) {
    quantize_row_q8_0(A + (size_t)i * k, Y + (size_t)i * nb, k);
    for (int r = 0; r < n; r++) ne_vec_dot_q4_0_q8_0(k, C + (size_t)i * n + r, Q + (size_t)r * nb, Y + (size_t)i * nb);
  }
  int meta[3] = {n, k, m};
  dump(cs, "meta", "i4", meta, 4, 3);
  dump(cs, "W", "f4", W, 4, (size_t)n * k);
  dump(cs, "q4_0", "u1", Q, 1, sizeof(block_q4_0) * n * nb);
  dump(cs, "deq", "f4", D, 4, (size_t)n * k);
  dump(cs, "A", "f4", A, 4, (size_t)m * k);
  dump(cs, "q8_0", "u1", Y, 1, sizeof(block_q8_0) * m * nb);
  dump(cs, "C", "f4", C, 4, (size_t)m * n);
  free(W);
  free(Q);
  free(D);
  free(A);
  free(Y);
  free(C);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  for (int i = 0; i < (1 << 16); ++i) {  // ne_init (ne_layers.c:738-742)
    uint16_t ui = (uint16_t)i;
    ne_fp16_t ii;
    memcpy(&ii, &ui, sizeof(ii));
    table_f32_f16[i] = NE_COMPUTE_FP16_TO_FP32(ii);
  }
  g_dir = argv[1];
  char path[1024];
  snprintf(path, sizeof(path), "%s/manifest.txt", g_dir);
  g_man = fopen(path, "w");
  if (!g_man) return 3;
  case_q4_0("q4_0_n40_k256", 40, 256, 3, 1.f);
  case_q4_0("q4_0_n16_k1024", 16, 1024, 2, 0.05f);
  fclose(g_man);
  return 0;
}
