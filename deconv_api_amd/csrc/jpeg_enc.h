// Host-side baseline JPEG encoder and data-URL builder (jpeg_enc.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace dvjpeg {

// RGB uint8 HxWx3 -> baseline JFIF JPEG (YCbCr 4:2:0, IJG-scaled standard tables, quality 1..100);
// segments > 1 splits the scan with restart markers (independently encodable MCU-row groups)
std::string encode_jpeg(const uint8_t* rgb, int H, int W, int quality, int segments = 1);
// prefix + base64(jpeg) with urllib.parse.quote's escaping of '+' and '=' (reference quirk Q3)
std::string data_url(const std::string& jpeg, const std::string& prefix);
// B images encoded on `threads` native threads (call with the GIL released); with fewer images
// than threads each image is split into restart segments so one request also uses every thread
std::vector<std::string> encode_data_urls(const uint8_t* rgb, int B, int H, int W, int quality,
                                          const std::string& prefix, int threads);

// payload of a data URL (between the first and second comma) -> bytes, with CPython's non-strict
// base64.b64decode semantics and error messages; false + err on error (call with the GIL released)
bool data_url_b64decode(const char* uri, size_t n, std::string& out, std::string& err);

// Everything the GPU encoder (jpeg_gpu.hip) needs, laid out as its kernels read it: quantizer
// reciprocals in the AAN DCT's transposed coefficient layout, the zig-zag source map, and the
// Annex K Huffman codes (DC: 12 symbols, AC: 256) for luma (0) / chroma (1).
struct GpuTables {
  float rl[64], rc[64];
  uint8_t zz_src[64];
  uint16_t dc_code[2][12];
  uint8_t dc_len[2][12];
  uint16_t ac_code[2][256];
  uint8_t ac_len[2][256];
};
GpuTables gpu_tables(int quality);
// SOI .. SOS of the stream encode_jpeg writes for (H, W, quality) with a restart marker after every
// ``restart_rows`` MCU rows (0: none)
std::string jpeg_header(int H, int W, int quality, int restart_rows);
// B images from the GPU encoder: header + entropy-coded bytes [off[b], off[b+1]) + EOI, base64'd
// with the quote() escaping, on `threads` native threads (call with the GIL released)
std::vector<std::string> data_urls_from_scans(const std::string& header, const uint8_t* scans, const int64_t* off,
                                              int B, const std::string& prefix, int threads);

}  // namespace dvjpeg
