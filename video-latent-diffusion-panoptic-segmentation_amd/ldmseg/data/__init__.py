from .bitcodec import BitmapCodecMixin, decode_bitmap, encode_bitmap  # noqa: F401
