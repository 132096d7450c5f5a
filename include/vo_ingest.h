/*
 * vo_ingest.h -- host-side frame ingest for the MI355X VO path (libvo_ingest.so).
 *
 * Replaces the per-frame image reads of the reference driver, utils.py:55-81:
 *   cv2.imread(os.path.join(kitti_path, '05/image_0', f'{i:06d}.png'), cv2.IMREAD_GRAYSCALE)
 *   cv2.imread(os.path.join(parking_path, f'images/img_{i:05d}.png'), cv2.IMREAD_GRAYSCALE)
 * (Malaga's JPEGs are not decoded here.)  PNG decoding runs on a pool of host threads straight
 * into caller memory (pinned, so the host->HBM copy of one batch overlaps the decode of the next).
 * Status codes: 0 ok, -1 bad argument, -3 I/O, -4 unsupported format, -5 size mismatch, -6 zlib.
 */
#ifndef VO_INGEST_H
#define VO_INGEST_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* IHDR of an in-memory PNG: width, height, channels, bit depth. */
int vo_png_info(const uint8_t* data, size_t len, int* w, int* h, int* channels, int* depth);

/* cv2.imread(..., IMREAD_GRAYSCALE) of an in-memory PNG into out[h][pitch] (utils.py:59,81). */
int vo_png_decode_gray(const uint8_t* data, size_t len, uint8_t* out, int64_t pitch, int w, int h);

/* Decoder thread pool. */
void* vo_ingest_create(int n_threads);
void vo_ingest_destroy(void* pool);

/* Decode n PNG files (W x H each) into out + i * frame_stride; per-file codes in status. */
int vo_ingest_png_files(void* pool, const char* const* paths, int n, uint8_t* out, int64_t frame_stride,
                        int W, int H, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif
