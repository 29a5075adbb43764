"""Model families: GPT (headline: GPT-3 1.3B hybrid-parallel pretraining; serving via
inference.generation), BERT (pretraining / classification). Vision models live in
``paddle_infer_amd.vision.models``."""
from .gpt import (GPTConfig, GPTModel, GPTForPretraining, GPTPretrainingCriterion,  # noqa: F401
                  gpt_config, PRESETS)
from .bert import (BertConfig, BertModel, BertForPretraining,  # noqa: F401
                   BertForSequenceClassification, bert_config)
