"""Alias of src/s3od/utils.py."""
from s3od_amd.utils import get_pad_info, remove_padding  # noqa: F401
