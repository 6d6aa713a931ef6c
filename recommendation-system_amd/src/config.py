"""Environment-driven defaults (mirrors src/config.py of the reference, :1-47)."""
import os
from pathlib import Path

try:  # python-dotenv is optional here (reference: config.py:4-7)
    from dotenv import load_dotenv
except ImportError:  # pragma: no cover - absent in this image
    def load_dotenv(*_a, **_k):
        return False

load_dotenv()

BASE_DIR = Path(os.environ.get("HVAE_BASE_DIR", Path(__file__).resolve().parent.parent))


class Config:
    DATA_DIR = BASE_DIR / "data"
    RAW_DATA_FILE = os.getenv("RAW_DATA_FILE", "Toys_and_Games_5.jsonl")
    PROCESSED_DATA_FILE = os.getenv("PROCESSED_DATA_FILE", str(DATA_DIR / "processed_interactions.csv"))

    MODEL_DIR = BASE_DIR / "models"
    EMBEDDINGS_DIR = BASE_DIR / "embeddings"
    MODEL_FILE = os.getenv("MODEL_FILE", str(MODEL_DIR / "best_model.pth"))
    ENCODER_FILE = os.getenv("ENCODER_FILE", str(MODEL_DIR / "label_encoders.pkl"))
    EMBEDDINGS_FILE = os.getenv("EMBEDDINGS_FILE", str(EMBEDDINGS_DIR / "item_embeddings.npy"))

    BATCH_SIZE = int(os.getenv("BATCH_SIZE", 64))
    LEARNING_RATE = float(os.getenv("LEARNING_RATE", 1e-3))
    EPOCHS = int(os.getenv("EPOCHS", 10))
    LATENT_DIM = int(os.getenv("LATENT_DIM", 50))
    HIDDEN_DIM = int(os.getenv("HIDDEN_DIM", 256))

    # MI355X path knobs (not in the reference)
    PRECISION = os.getenv("HVAE_PRECISION", "")  # "", "bf16" or "fp32" (decoder MFMA dtype)

    @classmethod
    def ensure_dirs(cls):
        """Create data/ and models/ on demand (the reference does it at import, config.py:47)."""
        cls.DATA_DIR.mkdir(parents=True, exist_ok=True)
        cls.MODEL_DIR.mkdir(parents=True, exist_ok=True)


config = Config()
