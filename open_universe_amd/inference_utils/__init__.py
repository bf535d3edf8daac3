"""Drop-in inference API: ``load_model`` and ``add_enhance_arguments``."""
from .model_loader import load_model
from .signature_to_parser import add_enhance_arguments

__all__ = ["load_model", "add_enhance_arguments"]
