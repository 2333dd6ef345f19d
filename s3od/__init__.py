"""Drop-in alias of the reference's inference package (src/s3od/__init__.py:1-5):
``from s3od import BackgroundRemoval, RemovalResult`` resolves to the MI355X implementation."""
from s3od_amd.predictor import BackgroundRemoval, RemovalResult

__version__ = "0.1.0"
__all__ = ["BackgroundRemoval", "RemovalResult"]
