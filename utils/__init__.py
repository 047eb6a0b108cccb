"""Drop-in `utils` package.  Unlike the reference's utils/__init__.py (which eagerly imports
pycocoevalcap/pycocotools through eval_metrics and scst_loss), importing a submodule here pulls
in no third-party metric package."""
