from .blokus_wrapper import ColosseumBlokusGameWrapper

__all__ = ["ColosseumBlokusGameWrapper"]
