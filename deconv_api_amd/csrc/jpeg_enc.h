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

}  // namespace dvjpeg
