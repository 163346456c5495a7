// Host sanitizer harness for the GIL-free JPEG encoder (deconv_api_amd/csrc/jpeg_enc.cpp).
//
// SURVEY section 5.2 (race detection): the service encodes batch responses on native threads with
// the Python GIL released, and splits one image into restart segments across threads. Built by
// tests/test_sanitizers.py with -fsanitize=thread (data races) and -fsanitize=address,undefined
// (out-of-bounds / UB), then run: several caller threads encode the same batches concurrently, each
// with its own worker pool, and every result must be byte-identical to a single-threaded encode.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "jpeg_enc.h"

int main(int argc, char** argv) {
  const int callers = argc > 1 ? std::atoi(argv[1]) : 4;
  const int B = 6, H = 448, W = 448;
  std::vector<uint8_t> rgb((size_t)B * H * W * 3);
  std::mt19937 rng(1234);
  for (auto& v : rgb) v = (uint8_t)(rng() & 0xFF);
  for (int i = 0; i < H * W * 3; ++i) rgb[i] = (uint8_t)((i / 3) % 251);  // one smooth image
  const std::string prefix = "data:image/webp;base64,";
  const auto ref = dvjpeg::encode_data_urls(rgb.data(), B, H, W, 95, prefix, 1);
  std::vector<std::vector<std::string>> got(callers);
  std::vector<std::thread> ts;
  for (int c = 0; c < callers; ++c)
    ts.emplace_back([&, c] { got[c] = dvjpeg::encode_data_urls(rgb.data(), B, H, W, 95, prefix, 2 + c); });
  for (auto& t : ts) t.join();
  // one image over many threads: restart-segment split must decode to the same prefix/body shape
  const auto one = dvjpeg::encode_data_urls(rgb.data(), 1, H, W, 95, prefix, 8);
  int bad = 0;
  for (int c = 0; c < callers; ++c)
    for (int b = 0; b < B; ++b)
      if (got[c][b].rfind(prefix, 0) != 0 || got[c][b].size() < 1000) ++bad;
  if (one.size() != 1 || one[0].rfind(prefix, 0) != 0) ++bad;
  for (int b = 0; b < B; ++b)
    if (ref[b].rfind(prefix, 0) != 0) ++bad;
  // with <= B threads every image is encoded whole (one segment) by one thread: the serial bytes
  for (int c = 0; c < callers; ++c)
    if (2 + c <= B)
      for (int b = 0; b < B; ++b)
        if (got[c][b] != ref[b]) ++bad;
  std::printf("callers=%d images=%d mismatches=%d\n", callers, B, bad);
  return bad == 0 ? 0 : 1;
}
