/* Harness of oracle/sift_oracle.c for the sanitizer build (tests/test_sanitize.py; SURVEY.md
 * §5): reads (int32 w, int32 h, w*h gray bytes) from argv[1], runs sift_oracle_detect as
 * oracle/sift.py does (count, then keypoints + descriptors) and writes (int32 n, x, y, size,
 * angle, response [f32 n each], octave [i32 n], descriptors [f32 n*128]) to argv[2]. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int sift_oracle_detect(const uint8_t* gray, int w, int h, int L, double contrastThreshold,
                       double edgeThreshold, double sigma, int cap, float* kx, float* ky,
                       float* ksize, float* kangle, float* kresp, int* koct, float* desc);

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* in = fopen(argv[1], "rb");
  if (!in) return 2;
  int32_t wh[2];
  if (fread(wh, 4, 2, in) != 2 || wh[0] < 1 || wh[1] < 1 || wh[0] > 8192 || wh[1] > 8192) return 2;
  const size_t np = (size_t)wh[0] * wh[1];
  uint8_t* g = malloc(np);
  if (fread(g, 1, np, in) != np) return 2;
  fclose(in);
  const int n = sift_oracle_detect(g, wh[0], wh[1], 3, 0.04, 10.0, 1.6, 0, NULL, NULL, NULL,
                                   NULL, NULL, NULL, NULL);
  if (n < 0) return 3;
  float* f = calloc((size_t)n * 5 + 1, sizeof(float));
  int* oc = calloc((size_t)n + 1, sizeof(int));
  float* d = calloc((size_t)n * 128 + 1, sizeof(float));
  const int m = sift_oracle_detect(g, wh[0], wh[1], 3, 0.04, 10.0, 1.6, n, f, f + n, f + 2 * n,
                                   f + 3 * n, f + 4 * n, oc, d);
  if (m != n) return 4;
  FILE* out = fopen(argv[2], "wb");
  if (!out) return 2;
  fwrite(&n, 4, 1, out);
  fwrite(f, sizeof(float), (size_t)n * 5, out);
  fwrite(oc, sizeof(int), (size_t)n, out);
  fwrite(d, sizeof(float), (size_t)n * 128, out);
  fclose(out);
  free(g);
  free(f);
  free(oc);
  free(d);
  return 0;
}
