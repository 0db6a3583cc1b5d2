from .cli import cli, main
