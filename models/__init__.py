"""Drop-in `models` package: same exports as the reference's models/__init__.py:4-5."""
from .vit_transformer_model import ViTTransformerCaptioning, build_model as build_vit_model
from .grid_transformer_model import GridTransformerCaptioning, build_model as build_grid_model

__all__ = ["ViTTransformerCaptioning", "GridTransformerCaptioning", "build_vit_model", "build_grid_model"]
