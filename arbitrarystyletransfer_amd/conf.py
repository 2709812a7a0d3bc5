"""Configuration tables of the reference (conf.py), restated so `from models import *` callers
(train.py:15-16) find the same names. Values follow conf.py:3-113."""
import torch

device = "cuda" if torch.cuda.is_available() else "cpu"   # conf.py:3 (HIP device on ROCm)
img_sizes = [96, 128, 160]                                  # conf.py:4
imsize = 320 if torch.cuda.is_available() else 128          # conf.py:8

EXPAND_RATIO = 3                                            # conf.py:71
expand_ratios = [1, 6, 6, 6, 6, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4]
kernel_sizes = [3, 3, 3, 3, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5]

# (c_in, c_out, stride, kernel, expand_ratio), conf.py:75-91
enc_conv_shapes = [
    (3, 16, 1, 3, 1),
    (16, 16, 1, 3, 6),
    (16, 24, 2, 3, 6),
    (24, 24, 1, 3, 6),
    (24, 40, 2, 5, 6),
    (40, 40, 1, 5, 4),
    (40, 40, 1, 5, 4),
    (40, 80, 2, 3, 4),
    (80, 80, 1, 3, 4),
    (80, 80, 1, 3, 4),
    (80, 96, 1, 5, 4),
    (96, 96, 1, 5, 3),
    (96, 128, 1, 3, 3),
    (128, 128, 1, 3, 3),
    (128, 128, 1, 3, 3)]

# conf.py:93-109
decoder_conv_shapes = [
    (128, 128, 1, 3, 3),
    (128, 128, 1, 3, 3),
    (128, 96, 1, 3, 3),
    (96, 96, 1, 5, 3),
    (96, 80, 1, 5, 4),
    (80, 80, 1, 3, 4),
    (80, 80, 1, 3, 4),
    (80, 40, 1, 3, 4),
    (40, 40, 1, 5, 4),
    (40, 40, 1, 5, 4),
    (40, 24, 1, 5, 6),
    (24, 24, 1, 3, 6),
    (24, 16, 1, 3, 6),
    (16, 16, 1, 3, 6),
    (16, 3, 1)]

enc_out_layers = [12, 14]                                   # conf.py:112
enc_out_channels = 128                                      # conf.py:113

# dataset roots (conf.py:121-122); the data path is out of scope
content_dir = ["temp_dataset/content/"]
style_dir = ["temp_dataset/style/"]
