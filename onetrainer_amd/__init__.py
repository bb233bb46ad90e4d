"""onetrainer_amd: MI355X-native (gfx950) diffusion training step behind OneTrainer's
modules/modelSetup + modules/trainer surface.  See DESIGN.md."""
__version__ = "0.1.0"
