"""serving"""
