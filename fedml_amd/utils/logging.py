"""Logger factory (reference: `utils/logging.py:12-33`)."""
import logging
import sys


class LoggerCreator:
    @staticmethod
    def create_logger(name=None, level=logging.INFO, args=None):
        logger = logging.getLogger(name)
        logger.setLevel(level)
        if not logger.handlers:
            rank = getattr(args, "rank", 0) if args is not None else 0
            h = logging.StreamHandler(sys.stdout)
            h.setFormatter(logging.Formatter(f"[rank {rank}] %(asctime)s %(levelname)s %(filename)s:%(lineno)d %(message)s"))
            logger.addHandler(h)
        return logger
