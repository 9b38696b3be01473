"""sdface-gan_amd: MI355X-native SDF + hash-grid renderer for SDFace-GAN.

Import name: ``sdface_gan_amd`` (see ``sdfr_loader.py`` at the repository root;
the directory name is not a valid Python identifier).

Drop-in surface (reference: im2scene/sdf/models/):
  Generator, VolumeFeatureRenderer, NGPSIRENGenerator, SirenGenerator,
  FCGenerator, LinearLayer, FiLMSiren, get_encoder      (sdf_model.py)
  GridEncoder, grid_encode                              (gridencoder/grid.py)
  SHEncoder, sh_encode                                  (shencoder/sphere_harmonics.py)
  generate_camera_params                                (sdf_utils.py:97-159)
  align_volume, extract_mesh_with_marching_cubes (+ marching_cubes, Mesh:
  HIP, csrc/mesh.hip), xyz2mesh                       (sdf_utils.py:164-223)
  SDFOptions, vol_render_opt                            (sdf_utils.py:447, training_utils.py:144)
Beyond the reference: GraphedGenerator (HIP-graph replay of the inference forward).
"""
from . import _lib  # noqa: F401
from .camera import generate_camera_params  # noqa: F401
from .encoders import GridEncoder, SHEncoder, grid_encode, sh_encode  # noqa: F401
from . import decoder_ops  # noqa: F401
from .generator import (Blur, Decoder, EqualLinear, FusedLeakyReLU, Generator,  # noqa: F401
                        MappingLinear, ModulatedConv2d, NoiseInjection, PixelNorm, StyledConv,
                        ToRGB, Upsample, fused_leaky_relu, make_kernel, upfirdn2d)
from .graphs import GraphedGenerator  # noqa: F401
from .mesh import (Mesh, align_volume, extract_mesh_with_marching_cubes,  # noqa: F401
                   marching_cubes, xyz2mesh)
from .options import AttrDict, SDFOptions, vol_render_opt  # noqa: F401
from . import training  # noqa: F401  (stage-2 DDP trainer, Discriminator, losses)
from .renderer import (FCGenerator, FiLMSiren, LinearLayer, NGPSIRENGenerator,  # noqa: F401
                       SirenGenerator, VolumeFeatureRenderer, get_encoder)

__version__ = "0.1.0"
