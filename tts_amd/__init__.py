"""tts_amd — MI355X-native Tacotron2-DDC + MultiBand-MelGAN inference path.

Drop-in replacements for the reference's hot-path modules; compute runs in the HIP library
``tts_amd/libttship.so`` (C ABI: ``include/ttship.h``).
"""

from .factories import AttrDict, load_config, setup_generator, setup_model  # noqa: F401
from .glow_tts import GlowTts  # noqa: F401
from .speaker_encoder import SpeakerEncoder  # noqa: F401
from .tacotron2 import Tacotron2  # noqa: F401
from .vocoder import (FullbandMelganGenerator, MelganGenerator, MultibandMelganGenerator, ParallelWaveganGenerator,  # noqa: F401
                      PQMF)

__version__ = "0.1.0"
