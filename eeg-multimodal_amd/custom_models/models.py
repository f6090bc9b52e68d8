"""Drop-in for python/src/custom_models/models.py: the paper's feature-level Laplacian-dropout models
with the reference's constructor and forward(eeg_*, eeg_mask, act_*, act_mask, epsilon, hard)
signatures, on the HIP engine:

  TICA_LapDropout  models.py:28-82    EEG text (BERT) + action image, cross-attention decoder
  TTCA_LapDropout  models.py:84-129   EEG text + action text (one BERT), sequence decoder
  ITCA_LapDropout  models.py:130-175  EEG image + action text, cross-attention decoder
  IICA_LapDropout  models.py:176-214  EEG image + action image, decoder over one memory token
  TISC_LapDropout  models.py:215-272  EEG text + action image, 2-token TransformerEncoder
  TICA_NonPrivate  models.py:309-352  TICA without the privacy stage (base_train's 'NDP' baseline)

The two remaining comparison baselines are importable (base_train.py:7 imports every name) but not
built — they are other experiments' models, outside the fusion step — and raise on
construction:
  TICA_DPSGD                models.py:274-307  a two-feature (1536-d) fusion without the decoder
  TISC_LapDropoutEquWeight  models.py:354-408  feature Dropout(rate) + one Laplace(0, 1/eps_hat) per row
"""
from eegfusion.modules import (IICA_LapDropout, ITCA_LapDropout, TICA_LapDropout, TICA_NonPrivate,  # noqa: F401
                               TISC_LapDropout, TTCA_LapDropout)


class _NotBuilt:
    ref = ""

    def __init__(self, *a, **k):
        raise NotImplementedError(
            f"{type(self).__name__} ({self.ref}) is a comparison baseline outside the fusion training path this "
            "build implements (DESIGN.md §9); use TICA_LapDropout / TICA_NonPrivate or the reference's own model")


class TICA_DPSGD(_NotBuilt):
    ref = "python/src/custom_models/models.py:274-307"


class TISC_LapDropoutEquWeight(_NotBuilt):
    ref = "python/src/custom_models/models.py:354-408"
