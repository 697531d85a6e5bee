"""MI355X-native QGMAP optical flow (drop-in for gqmap_gpu_mixture.m /
gqmap_gpuSuper_mix_entropy.m).  The compute lives in libgqmap.so (HIP,
gfx950); this package is the host-side mirror of the reference's call
interface and driver scripts."""
from .engine import (Engine, State, aepe, comm_unique_id, gqmap_gpu_mixture, gqmap_gpuSuper_mix_entropy,
                     initial_state, make_options, rand_uniform, strip_split, tile_group_run)
from .flowio import load_pair, load_preprocessed, read_flow_file, rgb2gray, write_flow_file
from .ops import flow_to_color, gauss_hermite, imresize, mixture_map, projsplx, resize_len, warp_image
from .legacy import gqmap_cpu, gqmap_cpu_device
from .pyramid import C3_SCALES, REFERENCE_SCALES, Pyramid, ctf_options, gqmap_ctf, optical_flow_ctf

__all__ = ["Engine", "State", "aepe", "gqmap_gpu_mixture", "gqmap_gpuSuper_mix_entropy",
           "initial_state", "make_options", "rand_uniform", "load_pair", "load_preprocessed", "read_flow_file",
           "rgb2gray", "write_flow_file", "flow_to_color", "gauss_hermite", "mixture_map",
           "projsplx", "imresize", "resize_len", "warp_image", "Pyramid", "gqmap_ctf",
           "optical_flow_ctf", "ctf_options", "C3_SCALES", "REFERENCE_SCALES", "comm_unique_id",
           "tile_group_run", "strip_split", "gqmap_cpu", "gqmap_cpu_device"]
