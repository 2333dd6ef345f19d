"""Alias of src/s3od/model.py's public class."""
from s3od_amd.model import DPTSegmentation  # noqa: F401
