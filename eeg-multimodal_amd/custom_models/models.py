"""Drop-in for python/src/custom_models/models.py: the paper's feature-level Laplacian-dropout models
with the reference's constructor and forward(eeg_*, eeg_mask, act_*, act_mask, epsilon, hard)
signatures, on the HIP engine:

  TICA_LapDropout  models.py:28-82    EEG text (BERT) + action image, cross-attention decoder
  TTCA_LapDropout  models.py:84-129   EEG text + action text (one BERT), sequence decoder
  ITCA_LapDropout  models.py:130-175  EEG image + action text, cross-attention decoder
  IICA_LapDropout  models.py:176-214  EEG image + action image, decoder over one memory token
  TISC_LapDropout  models.py:215-272  EEG text + action image, 2-token TransformerEncoder
"""
from eegfusion.modules import (IICA_LapDropout, ITCA_LapDropout, TICA_LapDropout, TISC_LapDropout,  # noqa: F401
                               TTCA_LapDropout)
