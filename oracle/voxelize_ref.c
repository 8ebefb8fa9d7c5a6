/*
 * PARITY ORACLE — TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product path never does.
 *
 * CPU restatement of mmcv `hard_voxelize_forward_cpu` (mmcv>=2.0.0, requirements.txt:8;
 * upstream mmcv/ops/csrc/pytorch/cpu/voxelization.cpp, `hard_voxelize_forward_cpu_kernel`),
 * the op behind upstream mmdet3d Det3DDataPreprocessor.voxelize for the voxel_layer of
 * configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py:48-53.
 * mmcv is not in this container; the algorithm restated from its public
 * source, single-threaded, in point order:
 *
 *   for each point i:
 *     for each axis j (x, y, z):  c = floor((p[j] - range_min[j]) / voxel_size[j])  [float32]
 *                                 reject the point if c < 0 || c >= grid[j]
 *                                 coor[2 - j] = c            (coors stored z, y, x)
 *     voxelidx = coor_to_voxelidx[coor]
 *     if voxelidx == -1:  if voxel_num >= max_voxels: skip point
 *                         voxelidx = voxel_num++; record coors[voxelidx]
 *     if num_points[voxelidx] < max_points: voxels[voxelidx][num] = p; num_points++
 *
 * grid[j] = round((range_max[j] - range_min[j]) / voxel_size[j]) in float32.
 * The dense coor_to_voxelidx grid is replaced by an open-addressing hash (same result).
 * Non-finite coordinates are rejected (mmcv leaves int(floor(NaN)) undefined).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_hard_voxelize(const float* pts, int n, int F, const float* vs, const float* rng,
                         int max_points, int max_voxels, float* voxels, int* coors, int* npts) {
  int grid[3];
  for (int j = 0; j < 3; ++j) {
    float span = rng[3 + j] - rng[j];
    grid[j] = (int)roundf(span / vs[j]);
  }
  size_t cap = 1;
  while (cap < (size_t)2 * (size_t)(n > 0 ? n : 1)) cap <<= 1;
  int64_t* hkey = (int64_t*)malloc(cap * sizeof(int64_t));
  int* hval = (int*)malloc(cap * sizeof(int));
  if (!hkey || !hval) { free(hkey); free(hval); return -1; }
  for (size_t k = 0; k < cap; ++k) hkey[k] = -1;
  memset(voxels, 0, sizeof(float) * (size_t)max_voxels * max_points * F);
  memset(npts, 0, sizeof(int) * (size_t)max_voxels);
  int voxel_num = 0;
  for (int i = 0; i < n; ++i) {
    const float* p = pts + (size_t)i * F;
    int c[3];
    int failed = 0;
    for (int j = 0; j < 3; ++j) {
      float cf = floorf((p[j] - rng[j]) / vs[j]);
      if (!(cf >= 0.0f && cf < (float)grid[j])) { failed = 1; break; }
      c[2 - j] = (int)cf;
    }
    if (failed) continue;
    int64_t key = ((int64_t)c[0] * grid[1] + c[1]) * grid[0] + c[2];
    size_t h = (size_t)((uint64_t)key * 0x9E3779B97F4A7C15ull) & (cap - 1);
    while (hkey[h] != -1 && hkey[h] != key) h = (h + 1) & (cap - 1);
    int vid;
    if (hkey[h] == -1) {
      if (voxel_num >= max_voxels) continue;
      vid = voxel_num++;
      hkey[h] = key;
      hval[h] = vid;
      coors[vid * 3 + 0] = c[0];
      coors[vid * 3 + 1] = c[1];
      coors[vid * 3 + 2] = c[2];
    } else {
      vid = hval[h];
    }
    int num = npts[vid];
    if (num < max_points) {
      memcpy(voxels + ((size_t)vid * max_points + num) * F, p, sizeof(float) * F);
      npts[vid] = num + 1;
    }
  }
  free(hkey);
  free(hval);
  return voxel_num;
}
