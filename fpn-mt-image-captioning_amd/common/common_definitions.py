"""Hyper-parameters of the captioning model, same names and defaults as the
reference's common/common_definitions.py:6-70 (TF objects replaced by names).

Additions for the MI355X build (no reference counterpart):
  BACKBONE        - FeatureExtractor backbone ('resnet50' | 'resnet101'); the
                    reference hard-codes MobileNetV2 (models/retinanet.py:274)
                    but every benchmarked config (BASELINE.json) names ResNet-FPN.
  COMPUTE_DTYPE   - 'bf16' (MFMA bf16, fp32 accumulate) or 'fp32' (exact f32
                    MFMA, parity mode).
  CLIPNORM_MODE   - 'per_tensor' (TF >= 2.4 OptimizerV2 clip_by_norm per
                    gradient, IndexedSlices norm for the embedding) or 'none'
                    (TF 2.0-2.3 custom loops ignored clipnorm); SURVEY App. A #13.
"""
import logging

IS_TRAINING = True
USE_GPU = True
LOGGING_LEVEL = logging.INFO

TOP_K = 10000  # tokenizer vocabulary (target_vocab_size)

ACTIVATION = "leaky_relu"  # tf.nn.leaky_relu, alpha = 0.2
LEAKY_ALPHA = 0.2
KERNEL_INITIALIZER = "he_normal"

IMAGE_INPUT_SIZE = 512
BATCH_SIZE = 10
BUFFER_SIZE = 1000
EPOCHS = 100
BEAM_SEARCH_N = 4
N_VAL_DATASET = 50
N_TRAIN_DATASET = None
N_EPOCH_TO_EVALUATE = 1
AMOUNT_OF_VALIDATION = 100
DROPOUT_RATE = 0.1

MIN_EPOCH_TO_BREAK = EPOCHS // 2
GAP_OF_DEAD_EPOCH = 25
WARM_UP_STEPS = 4000

DATADIR = "datasets/iuxray"
DATATYPE_VAL = "val2017"
DATATYPE_TRAIN = "train2017"

TOKENIZER_FILENAME = "datasets/_tokenizer.json"
ADDITIONAL_FILENAME = "datasets/_additional_extractor.json"
RETINANET_WEIGHT_PATH = None  # the reference's h5 (model_weights/...) is not shipped
TRANSFORMER_WEIGHT_PATH = None
TRANSFORMER_CHECKPOINT_PATH = "./checkpoints/train/multimodal_transformer"
RESULT_FILE = "results/" + DATATYPE_VAL + "_captions_result.json"

num_layers = 6
d_model = 512
dff = 2048
num_heads = 8

NUM_OF_CLASSES = 80
NUM_OF_RETINANET_FILTERS = 256
NUM_OF_ANCHORS = 9
NUM_OF_PYRAMIDS = 5
N_CONV_SUBMODULE = 2

BASELINE_INDEX = 3

# --- MI355X build additions --------------------------------------------
BACKBONE = "resnet50"
COMPUTE_DTYPE = "bf16"
CLIPNORM_MODE = "per_tensor"
START_TOKEN = 2  # '<start>' id in the synthetic tokenizer
END_TOKEN = 3    # '<end>'

logging.basicConfig(level=LOGGING_LEVEL)
