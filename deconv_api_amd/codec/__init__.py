from .image import (DATA_URL_PREFIX, ImageDecodeError, decode_image, encode_data_url, encode_data_urls, encode_jpeg,
                    encode_jpeg_pil, make_data_url, parse_result_data_url, read_data_url, to_data_url)
from .pool import CodecPool

__all__ = ["DATA_URL_PREFIX", "ImageDecodeError", "decode_image", "encode_data_url", "encode_data_urls", "encode_jpeg",
           "encode_jpeg_pil", "make_data_url",
           "parse_result_data_url", "read_data_url", "to_data_url", "CodecPool"]
