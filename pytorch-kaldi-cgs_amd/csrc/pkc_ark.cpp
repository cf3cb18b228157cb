// pkc_ark.cpp — host-side Kaldi binary ark I/O for the chunk loader and the posterior writer.
//
// write: byte-compatible with the reference's data_io.write_mat (data_io.py:770-806):
//        "<key> \0B" "FM " '\4' <u32 rows> '\4' <u32 cols> <rows*cols f32 little endian>
// read : binary 'FM '/'DM ' matrices as produced by copy-feats (data_io.py:645-711); DM rows are
//        converted to f32 (the reference converts the whole chunk with .float() at core.py:94).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/pkc.h"

namespace pkc {
void set_error(const char* fmt, ...);
}

extern "C" int pkc_ark_write_mat(const char* path, int append, const char* key, int64_t rows,
                                 int64_t cols, const float* data) {
  if (!path || !key || rows < 0 || cols < 0 || (rows * cols > 0 && !data)) {
    pkc::set_error("pkc_ark_write_mat: bad arguments");
    return PKC_ERR_ARG;
  }
  FILE* f = fopen(path, append ? "ab" : "wb");
  if (!f) {
    pkc::set_error("pkc_ark_write_mat: cannot open %s", path);
    return PKC_ERR_IO;
  }
  const uint32_t r = (uint32_t)rows, c = (uint32_t)cols;
  const char four = 4;
  size_t ok = 1;
  if (key[0]) {
    ok &= fwrite(key, 1, strlen(key), f) == strlen(key);
    ok &= fwrite(" ", 1, 1, f) == 1;
  }
  ok &= fwrite("\0BFM ", 1, 5, f) == 5;
  ok &= fwrite(&four, 1, 1, f) == 1;
  ok &= fwrite(&r, 4, 1, f) == 1;
  ok &= fwrite(&four, 1, 1, f) == 1;
  ok &= fwrite(&c, 4, 1, f) == 1;
  if (rows * cols > 0) ok &= fwrite(data, sizeof(float), (size_t)(rows * cols), f) == (size_t)(rows * cols);
  if (fclose(f) != 0 || !ok) {
    pkc::set_error("pkc_ark_write_mat: write failed on %s", path);
    return PKC_ERR_IO;
  }
  return PKC_OK;
}

// offsets[i] = byte offset of matrix i's data; rows/cols; dtype folded into the sign of cols
// (cols < 0 means 'DM ' float64 data).  keys_buf receives NUL-separated keys.
extern "C" int64_t pkc_ark_index(const char* path, int64_t* offsets, int64_t* rows, int64_t* cols,
                                 int64_t cap, char* keys_buf, int64_t keys_cap) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    pkc::set_error("pkc_ark_index: cannot open %s", path);
    return PKC_ERR_IO;
  }
  int64_t n = 0, kpos = 0;
  std::vector<char> key;
  for (;;) {
    key.clear();
    int ch;
    while ((ch = fgetc(f)) != EOF && ch != ' ') key.push_back((char)ch);
    if (ch == EOF) break;
    while (!key.empty() && (key.back() == '\n' || key.back() == '\r')) key.pop_back();
    size_t s0 = 0;
    while (s0 < key.size() && (key[s0] == '\n' || key[s0] == '\r')) ++s0;
    unsigned char hdr[15];
    if (fread(hdr, 1, 15, f) != 15 || hdr[0] != 0 || hdr[1] != 'B' || hdr[5] != 4 || hdr[10] != 4) {
      fclose(f);
      pkc::set_error("pkc_ark_index: %s: unsupported matrix header (binary FM/DM only)", path);
      return PKC_ERR_UNSUPPORTED;
    }
    int esz;
    if (!memcmp(hdr + 2, "FM ", 3)) esz = 4;
    else if (!memcmp(hdr + 2, "DM ", 3)) esz = 8;
    else {
      fclose(f);
      pkc::set_error("pkc_ark_index: %s: compressed/unknown matrix type", path);
      return PKC_ERR_UNSUPPORTED;
    }
    int32_t r, c;
    memcpy(&r, hdr + 6, 4);
    memcpy(&c, hdr + 11, 4);
    const int64_t off = ftell(f);
    if (n < cap) {
      if (offsets) offsets[n] = off;
      if (rows) rows[n] = r;
      if (cols) cols[n] = esz == 4 ? c : -(int64_t)c;
      const int64_t kl = (int64_t)(key.size() - s0);
      if (keys_buf && kpos + kl + 1 <= keys_cap) {
        memcpy(keys_buf + kpos, key.data() + s0, (size_t)kl);
        keys_buf[kpos + kl] = 0;
        kpos += kl + 1;
      }
    }
    ++n;
    if (fseek(f, (long)((int64_t)r * c * esz), SEEK_CUR) != 0) break;
  }
  fclose(f);
  return n;
}

extern "C" int pkc_ark_read_rows(const char* path, int64_t offset, int64_t rows, int64_t cols,
                                 float* dst) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    pkc::set_error("pkc_ark_read_rows: cannot open %s", path);
    return PKC_ERR_IO;
  }
  if (fseek(f, (long)offset, SEEK_SET) != 0) {
    fclose(f);
    return PKC_ERR_IO;
  }
  const int64_t n = rows * (cols < 0 ? -cols : cols);
  size_t got;
  if (cols >= 0) {
    got = fread(dst, sizeof(float), (size_t)n, f);
  } else {
    std::vector<double> tmp((size_t)n);
    got = fread(tmp.data(), sizeof(double), (size_t)n, f);
    for (int64_t i = 0; i < n; ++i) dst[i] = (float)tmp[(size_t)i];
  }
  fclose(f);
  if ((int64_t)got != n) {
    pkc::set_error("pkc_ark_read_rows: short read on %s", path);
    return PKC_ERR_IO;
  }
  return PKC_OK;
}

// Kaldi CompressedMatrix "CM " (data_io.py:729-766, kaldi compressed-matrix.h): global header
// {min, range, rows, cols}, per-column uint16 percentiles {p0, p25, p75, p100} mapped to
// min + range * q / 65535, then cols x rows uint8 codes (column-major) decoded piecewise-linearly.
// Evaluated in float32 exactly as the reference's numpy expressions (no contraction into FMA).
extern "C" int64_t pkc_ark_cm_size(const unsigned char* blob, int64_t nbytes) {
  if (!blob || nbytes < 16) return PKC_ERR_ARG;
  int32_t rows, cols;
  memcpy(&rows, blob + 8, 4);
  memcpy(&cols, blob + 12, 4);
  if (rows < 0 || cols < 0) return PKC_ERR_ARG;
  return 16 + (int64_t)cols * 8 + (int64_t)rows * cols;
}

extern "C" int pkc_ark_decode_cm(const unsigned char* blob, int64_t nbytes, float* out) {
#pragma clang fp contract(off)
  const int64_t need = pkc_ark_cm_size(blob, nbytes);
  if (need < 0 || need > nbytes || !out) {
    pkc::set_error("pkc_ark_decode_cm: truncated or bad compressed matrix");
    return PKC_ERR_ARG;
  }
  float gmin, grange;
  int32_t rows, cols;
  memcpy(&gmin, blob, 4);
  memcpy(&grange, blob + 4, 4);
  memcpy(&rows, blob + 8, 4);
  memcpy(&cols, blob + 12, 4);
  const float scale = (float)1.52590218966964e-05;
  const unsigned char* ch = blob + 16;
  const unsigned char* data = ch + (int64_t)cols * 8;
  for (int32_t c = 0; c < cols; ++c) {
    float p[4];
    for (int q = 0; q < 4; ++q) {
      uint16_t v;
      memcpy(&v, ch + (int64_t)c * 8 + 2 * q, 2);
      float x = (float)v * grange;
      x = x * scale;
      p[q] = x + gmin;
    }
    const float s0 = (p[1] - p[0]) / 64.0f, s1 = (p[2] - p[1]) / 128.0f, s2 = (p[3] - p[2]) / 63.0f;
    for (int32_t r = 0; r < rows; ++r) {
      const unsigned b = data[(int64_t)c * rows + r];
      float v;
      if (b <= 64) v = p[0] + s0 * (float)b;
      else if (b > 192) v = p[2] + s2 * (float)(b - 192);
      else v = p[1] + s1 * (float)(b - 64);
      out[(int64_t)r * cols + c] = v;
    }
  }
  return PKC_OK;
}
