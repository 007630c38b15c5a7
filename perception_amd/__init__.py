"""perception_amd -- MI355X-native render-and-compare pose-search core (drop-in for the hot path of
Tacha-S/perception's PERCH 2.0 GPU path).  See DESIGN.md."""
__version__ = "0.1.0"
